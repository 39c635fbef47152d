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


def test_case_table_matches_oracle():
    """The kernel's generated table (csrc/case_table.h) agrees with the oracle's lower-casing on every
    accepted two-byte code point, and rejects exactly the non-1:1 ones."""
    import os
    import re

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    txt = open(os.path.join(root, "spark-text-clustering_amd", "csrc", "case_table.h")).read()
    body = txt[txt.index("{", txt.index("kLower2")) + 1:txt.index("};")]
    vals = [int(x, 16) for x in re.findall(r"0x[0-9A-Fa-f]+", body)]
    assert len(vals) == 0x700
    rejected = {cp for cp in range(0x100, 0x800) if vals[cp - 0x100] == 0}
    assert rejected == {0x130, 0x3A3, 0x23A, 0x23E}
    for cp in range(0x100, 0x800):
        if cp in rejected:
            continue
        assert O.java_lower(chr(cp)) == chr(vals[cp - 0x100]), hex(cp)
