"""CPU: the Tokenizer oracle (oracle.tokenize = [U] ml.feature.Tokenizer, toLowerCase.split("\\s"))
against the known answers of Java's String.split(regex) contract (limit 0: interior empty strings
kept, trailing ones removed, no match → the whole string) and Java's \\s class [ \\t\\n\\x0B\\f\\r].
No reference artifact holds tokenizer output (the reference tokenises with CoreNLP,
LDAClustering.scala:116-139), so these documented-behaviour vectors are what pins it."""
import pytest

from oracle import oracle as O

JAVA_SPLIT_KNOWN = [
    ("a b", ["a", "b"]),
    (" a", ["", "a"]),          # leading positive-width match keeps the empty piece
    ("a  b", ["a", "", "b"]),   # interior empty piece kept
    ("a ", ["a"]),              # trailing empty pieces removed
    ("a \t\n", ["a"]),
    ("", [""]),                 # no match: the input itself
    ("abc", ["abc"]),
    ("   ", []),                # every piece is a trailing empty
    ("\t\n\x0b\f\r ", []),
    ("x\x0by", ["x", "y"]),     # \x0B is in Java's \s
    ("x\u00a0y", ["x\u00a0y"]),  # NBSP is not (no UNICODE_CHARACTER_CLASS)
    ("x\u2003y", ["x\u2003y"]),  # nor EM SPACE
    ("x\x1cy", ["x\x1cy"]),     # nor the FS/GS/RS/US separators Python's str.split would take
]


@pytest.mark.parametrize("text,expected", JAVA_SPLIT_KNOWN)
def test_java_split_known_answers(text, expected):
    assert O.java_split_whitespace(text) == expected


def test_tokenize_lowercases_then_splits():
    assert O.tokenize("Hello  WORLD\tÄrger ÜBER Straße") == ["hello", "", "world", "ärger", "über", "straße"]
    assert O.tokenize("×ÞÀ") == ["×þà"]  # U+00D7 has no lower case


def test_java8_lower_known_answers():
    """Java 8 String.toLowerCase(Locale.ROOT) facts the oracle restates: Cyrillic/Greek/Armenian
    capitals map 1:1, Final_Sigma is contextual, İ expands, and code points Java 8 (Unicode 6.2)
    does not know stay as they are."""
    assert O.java_lower("МОСКВА Ёж ЇЖАК") == "москва ёж їжак"
    assert O.java_lower("ΟΔΟΣ Σ") == "οδος σ"          # final sigma at the word end, σ alone
    assert O.java_lower("İ") == "i̇"
    assert O.java_lower("Ϳ Ԩ") == "Ϳ Ԩ"              # U+037F, U+0528: Unicode 7.0 additions
    assert O.java_lower("ǅ Ǆ") == "ǆ ǆ"              # titlecase and capital digraph


def test_java8_lower_past_two_byte_code_points():
    """Three- and four-byte code points: Greek Extended, Latin Extended Additional, letterlike and
    enclosed capitals, fullwidth Latin, Glagolitic, Coptic, Deseret map 1:1; caseless characters such as
    U+2116 "№" stay; the Unicode 7.0+ / 8.0 cased additions Java 8 does not know (Cherokee capitals,
    Georgian Mtavruli, Latin Extended-D past U+A7AA, Osage, Adlam) stay as they are."""
    assert O.java_lower("ἈΘΗΝΑΙ Ἱ ὁ") == "ἀθηναι ἱ ὁ"
    assert O.java_lower("ḂẞẠ") == "ḃßạ"            # U+1E9E ẞ → ß (the kernel rejects it: 3 → 2 bytes)
    assert O.java_lower("ⅫⒶＡＺ") == "ⅻⓐａｚ"
    assert O.java_lower("ⰀⲀ") == "ⰰⲁ"
    assert O.java_lower("\U00010400\U00010427") == "\U00010428\U0001044f"
    assert O.java_lower("№ 2 ©") == "№ 2 ©"
    assert O.java_lower("ᎠᏴ") == "ᎠᏴ"                # Cherokee: caseless in Unicode 6.2
    assert O.java_lower("ᲐᲿ") == "ᲐᲿ"                # Georgian Mtavruli: Unicode 11.0
    assert O.java_lower("ꞫꞲꟂ") == "ꞫꞲꟂ"              # Latin Extended-D: Unicode 7.0–12.0
    assert O.java_lower("Ɦ") == "ɦ"                  # U+A7AA: Unicode 6.1, mapped (3 → 2 bytes: rejected)
    assert O.java_lower("\U000104B0\U0001E900") == "\U000104B0\U0001E900"  # Osage, Adlam


def _case_table():
    """csrc/case_table.h parsed back: {page: [256 entries]} for the pages that are not identity"""
    import os
    import re

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    txt = open(os.path.join(root, "spark-text-clustering_amd", "csrc", "case_table.h")).read()
    idx_body = txt[txt.index("{", txt.index("kCasePage[256]")) + 1:]
    idx = [int(x) for x in re.findall(r"-?\d+", idx_body[:idx_body.index("};")])]
    assert len(idx) == 256
    pages_body = txt[txt.index("kCasePages[kCasePagesN][256] = {") + 32:]
    pages_body = pages_body[:pages_body.index("\n};")]
    pages = re.findall(r"\{\s*// U\+([0-9A-F]{4})[^\n]*\n(.*?)\n\s*\}", pages_body, re.S)
    out = {}
    for start, body in pages:
        vals = [int(x, 16) for x in re.findall(r"0x[0-9A-Fa-f]+", body)]
        assert len(vals) == 256
        out[int(start, 16) >> 8] = vals
    # pages are emitted in code point order, page i + 1 of the index being the i-th emitted
    assert [idx[p] for p in out] == list(range(1, len(out) + 1)), "page index and page data disagree"
    assert sum(1 for i in idx if i) == len(out)
    return out


def test_case_table_matches_oracle():
    """The kernel's generated table (csrc/case_table.h) agrees with the oracle's Java 8 lower-casing on
    every BMP code point it maps (identity pages included), and leaves exactly the non-1:1 ones to rule
    (entry 0): İ (SpecialCasing), Σ (Final_Sigma) and the capitals whose lower case has another UTF-8
    length, whose rule table (kSpecialFrom / kSpecialTo) matches the oracle too."""
    pages = _case_table()
    expected_rejects = {0x130, 0x3A3, 0x23A, 0x23E, 0x1E9E, 0x2126, 0x212A, 0x212B, 0x2C62, 0x2C64, 0x2C6D,
                        0x2C6E, 0x2C6F, 0x2C70, 0x2C7E, 0x2C7F, 0xA78D, 0xA7AA}
    rejected = set()
    for cp in range(0x80, 0x10000):
        if 0xD800 <= cp <= 0xDFFF:
            continue
        ent = pages[cp >> 8][cp & 0xFF] if (cp >> 8) in pages else cp
        if ent == 0:
            rejected.add(cp)
            continue
        assert O.java_lower(chr(cp)) == chr(ent), hex(cp)
    assert rejected == expected_rejects
    special = _special_table()
    assert set(special) == expected_rejects - {0x130, 0x3A3}
    for cp, lc in special.items():
        assert O.java_lower(chr(cp)) == chr(lc), hex(cp)
    assert O.java_lower("\u0130") == "i\u0307"


def _generated(name):
    import os
    import re

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    txt = open(os.path.join(root, "spark-text-clustering_amd", "csrc", "case_table.h")).read()
    body = txt[txt.index("{", txt.index(name)) + 1:]
    return [int(x, 0) for x in re.findall(r"0x[0-9A-Fa-f]+|\b\d+\b", body[:body.index("};")])]


def _special_table():
    return dict(zip(_generated("kSpecialFrom["), _generated("kSpecialTo[")))


def test_final_sigma_classes_match_oracle():
    """case_table.h's Final_Sigma classes (0 other, 1 case-ignorable, 2 cased) decide Σ exactly as the
    oracle's lower-casing does: for every class-1/2 code point c and a sample of class-0 ones, ΑΣc and
    ΑΣcΒ lower-case to what the class predicts."""
    idx = _generated("kSigPage[")
    assert len(idx) == 4352
    import re
    import os

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    txt = open(os.path.join(root, "spark-text-clustering_amd", "csrc", "case_table.h")).read()
    body = txt[txt.index("kSigPages[kSigPagesN][64] = {") + 30:]
    pages = [[int(x, 16) for x in re.findall(r"0x[0-9A-F]{2}", row)] for row in re.findall(r"\{([^}]*)\}", body[:body.index("\n};")])]
    assert all(len(p) == 64 for p in pages) and len(pages) == max(idx)

    def cls(cp):
        pg = idx[cp >> 8]
        return (pages[pg - 1][(cp & 0xFF) >> 2] >> (2 * (cp & 3))) & 3 if pg else 0

    sample = [cp for cp in range(0x110000) if cls(cp)] + list(range(0x20, 0x80)) + list(range(0x3000, 0x3100))
    for cp in sample:
        if 0xD800 <= cp <= 0xDFFF:
            continue
        c = cls(cp)
        a = O.java_lower("\u0391\u03a3" + chr(cp))[1]
        b = O.java_lower("\u0391\u03a3" + chr(cp) + "\u0392")[1]
        want = {0: ("\u03c2", "\u03c2"), 1: ("\u03c2", "\u03c3"), 2: ("\u03c3", "\u03c3")}[c]
        assert (a, b) == want, (hex(cp), c, a, b)


def test_reference_book_slices_hold_the_round2_rejects():
    """tests/golden/books_text.json carries slices of every book line the round-2 kernel rejected
    (Walden's Greek Extended letters, four "№" lines) — no slice of the fixture is filtered."""
    from helpers import golden_json

    books = golden_json("books_text.json")
    joined = "".join(t["text"] for t in books["targets"])
    assert "\u1f31" in joined and "\u1f41" in joined and joined.count("\u2116") >= 4
