"""Generate spark-text-clustering_amd/csrc/case_table.h: Java 8 String.toLowerCase (root locale) for every
BMP code point, as the tokenizer kernel (K0) applies it.

    python tools/gen_case_table.py

Two levels: kCasePage[cp >> 8] is 0 for a page every code point of which maps to itself, else 1 + the
index of its 256-entry page in kCasePages, whose entry cp & 0xFF is the lower-case code point, or 0 when
the kernel must reject the character (STC_ERR_INVALID_ARG) because Java's mapping is not a same-length
1:1 code point map:
  * U+0130 İ → "i̇" (two code points, SpecialCasing),
    (U+0000's entry is 0 as well: the kernel maps ASCII itself and never looks it up)
  * U+03A3 Σ → σ or ς by context (Final_Sigma),
  * any capital whose lower case has another UTF-8 length (U+023A → U+2C65, U+1E9E ẞ → ß, U+2126 Ω → ω,
    U+212A K → k, U+2C62 Ɫ → ɫ, …).
Supplementary code points: Java 8 lower-cases only Deseret (U+10400–U+10427 → +0x28, done inline by
the kernel); everything else there is passed through.

Spark 2.4.3 runs on Java 8 (Unicode 6.2).  Python's database is newer (3.10: Unicode 13.0), so the
code points that gained a lower-case mapping after 6.2 map to themselves here, as Java 8 leaves
unassigned (and then caseless) characters unchanged: the cased additions of Unicode 7.0–13.0 (U+037F,
U+0528–U+052F, U+A698–U+A69F, U+A794–U+A79F, U+A7AB–U+A7FF, Georgian Mtavruli U+1C90–U+1CBF) and the
Cherokee letters U+13A0–U+13FF, caseless in 6.2 and given lower-case partners in 8.0.  Case pairs are
otherwise stable across versions (Unicode's case-pair stability policy), so Python's mapping is Java 8's
for everything else.  oracle/oracle.py holds the same set (tests/test_tokenizer_oracle.py checks the
generated table against it code point by code point).
"""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "spark-text-clustering_amd", "csrc", "case_table.h")

JAVA8_IDENTITY_RANGES = [(0x37F, 0x37F), (0x528, 0x52F), (0x13A0, 0x13FF), (0x1C90, 0x1CBF), (0xA698, 0xA69F),
                         (0xA794, 0xA79F), (0xA7AB, 0xA7FF)]


def java8_identity(cp):
    return any(lo <= cp <= hi for lo, hi in JAVA8_IDENTITY_RANGES)


def utf8_len(cp):
    return 1 if cp < 0x80 else 2 if cp < 0x800 else 3 if cp < 0x10000 else 4


def lower_entry(cp):
    """the table entry for a BMP code point: its lower-case code point, or 0 = reject"""
    if 0xD800 <= cp <= 0xDFFF or java8_identity(cp):
        return cp
    lc = chr(cp).lower()
    if cp == 0x3A3 or len(lc) != 1 or utf8_len(ord(lc)) != utf8_len(cp):
        return 0
    return ord(lc)


def special_maps():
    """the length-changing 1:1 maps among the rejected entries: {cp: lower cp} (İ and Σ are handled by rule)"""
    out = {}
    for cp in range(0x80, 0x10000):
        if 0xD800 <= cp <= 0xDFFF or java8_identity(cp) or cp in (0x130, 0x3A3):
            continue
        lc = chr(cp).lower()
        if len(lc) == 1 and utf8_len(ord(lc)) != utf8_len(cp):
            out[cp] = ord(lc)
    return out


# Final_Sigma (U+03A3 → ς when preceded by a cased letter, case-ignorables between, and not followed by
# case-ignorables then a cased letter): the class of every code point the rule's two scans look at, as
# Python's str.lower() — the oracle's lower-casing — applies it: 1 = case-ignorable (skipped), 2 = cased and
# not case-ignorable (ends a scan, counts), 0 = anything else (ends a scan).  Read off str.lower() itself
# ("AΣc" and "AΣcB"), so the table and the oracle cannot disagree.  Java 8's unassigned code points (the
# identity ranges) are class 0, as the oracle's per-segment lowering treats them.
SIG_OTHER, SIG_IGNORABLE, SIG_CASED = 0, 1, 2


def sigma_class(cp):
    if 0xD800 <= cp <= 0xDFFF or java8_identity(cp) or any(lo <= cp <= hi for lo, hi in SUPP_IDENTITY_RANGES):
        return SIG_OTHER
    c = chr(cp)
    a, b = ("A\u03a3" + c).lower()[1], ("A\u03a3" + c + "B").lower()[1]
    if a == "\u03c2" and b == "\u03c3":
        return SIG_IGNORABLE
    return SIG_CASED if a == "\u03c3" else SIG_OTHER


SUPP_IDENTITY_RANGES = [(0x104B0, 0x104FF), (0x10C80, 0x10CFF), (0x118A0, 0x118FF), (0x16E40, 0x16E9F),
                        (0x1E900, 0x1E95F)]


def sigma_pages():
    idx, data = [], []
    for p in range(0x110000 >> 8):
        cls = [sigma_class(cp) for cp in range(p << 8, (p + 1) << 8)]
        if not any(cls):
            idx.append(0)
            continue
        packed = [sum(cls[4 * i + j] << (2 * j) for j in range(4)) for i in range(64)]
        data.append(packed)
        idx.append(len(data))
    return idx, data


def pages():
    idx, data = [], []
    for p in range(256):
        ent = [lower_entry(cp) for cp in range(p << 8, (p + 1) << 8)]
        if all(e == (p << 8) + i for i, e in enumerate(ent)):
            idx.append(0)
        else:
            data.append(ent)
            idx.append(len(data))
    return idx, data


def main():
    idx, data = pages()
    rows = []
    for pi, ent in enumerate(data):
        page = idx.index(pi + 1)
        rows.append(f"    {{  // U+{page << 8:04X}–U+{(page << 8) + 255:04X}")
        for i in range(0, 256, 12):
            rows.append("        " + ", ".join(f"0x{x:04X}" for x in ent[i:i + 12]) + ",")
        rows.append("    },")
    irows = ["    " + ", ".join(f"{x:2d}" for x in idx[i:i + 16]) + "," for i in range(0, 256, 16)]
    n_rej = sum(1 for ent in data for e in ent if e == 0) - 1  # U+0000's entry (ASCII never looks it up)
    n_map = sum(1 for pi, ent in enumerate(data) for i, e in enumerate(ent)
                if e and e != (idx.index(pi + 1) << 8) + i)
    sp = special_maps()
    sidx, sdata = sigma_pages()
    assert len(sdata) < 256
    srows = ["    {" + ", ".join(f"0x{x:02X}" for x in ent) + "}," for ent in sdata]
    sirows = ["    " + ", ".join(f"{x:2d}" for x in sidx[i:i + 32]) + "," for i in range(0, len(sidx), 32)]
    special = ("// the capitals whose lower case has another UTF-8 length (their kCasePages entry is 0): cp → lower\n"
               f"constexpr int kSpecialN = {len(sp)};\n"
               "__device__ const uint16_t kSpecialFrom[kSpecialN] = {" + ", ".join(f"0x{k:04X}" for k in sp) + "};\n"
               "__device__ const uint16_t kSpecialTo[kSpecialN] = {" + ", ".join(f"0x{v:04X}" for v in sp.values()) + "};\n\n"
               "// Final_Sigma classes (2 bits per code point, 0 other, 1 case-ignorable, 2 cased), two levels over\n"
               "// U+0000–U+10FFFF: kSigPage[cp >> 8] = 0 (all other) or 1 + the page in kSigPages\n"
               f"constexpr int kSigPagesN = {len(sdata)};\n"
               "__device__ const uint8_t kSigPage[4352] = {\n" + "\n".join(sirows) + "\n};\n"
               "__device__ const uint8_t kSigPages[kSigPagesN][64] = {\n" + "\n".join(srows) + "\n};\n\n")
    txt = ("// case_table.h — GENERATED by tools/gen_case_table.py (do not edit): Java 8 String.toLowerCase\n"
           "// (root locale) of every BMP code point, two levels: kCasePage[cp >> 8] = 0 (the page maps to itself)\n"
           "// or 1 + its page in kCasePages, whose entry cp & 0xFF = the lower-case code point, 0 = rejected (see\n"
           f"// the generator for the rules).  {n_map} mapped, {n_rej} rejected.  Used by tokenizer.hip (K0).\n"
           "#pragma once\n#include <cstdint>\n\nnamespace stc {\nnamespace tokenizer {\n\n"
           f"constexpr int kCasePagesN = {len(data)};\n"
           "__device__ const uint8_t kCasePage[256] = {\n" + "\n".join(irows) + "\n};\n"
           "__device__ const uint16_t kCasePages[kCasePagesN][256] = {\n" + "\n".join(rows) + "\n};\n\n"
           + special +
           "}  // namespace tokenizer\n}  // namespace stc\n")
    open(OUT, "w").write(txt)
    print(f"wrote {OUT}: {len(data)} pages, {n_map} mapped, {n_rej} rejected")


if __name__ == "__main__":
    main()
