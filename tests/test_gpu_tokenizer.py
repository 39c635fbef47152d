"""GPU parity: the Tokenizer kernel K0 ([U] ml.feature.Tokenizer, toLowerCase.split("\\s")) through
the C ABI vs the oracle, bit-exact on tokens; Tokenizer → HashingTF fused on device vs oracle
tokenize + hashing_tf."""
import numpy as np
import pytest

from test_tokenizer_oracle import JAVA_SPLIT_KNOWN

pytestmark = pytest.mark.gpu

_ALPHABET = list("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789.,;'\"-") + \
    ["Ä", "Ö", "Ü", "ß", "é", "È", "Ç", "×", "Þ", "µ", "\u00a0", "—", "“", "”", "€", "漢", "字", "😀",
     "Ж", "ж", "Ё", "Ї", "Ґ", "Ω", "ς", "Ğ", "Ł", "Ŋ", "Ǆ", "ǅ", "Ա", "Ͳ", "Ϳ", "Ԩ", "\u0301", "א", "ب",
     # three- and four-byte: Greek Extended, Latin Extended Additional, letterlike / enclosed / fullwidth
     # capitals, Glagolitic, Coptic, Georgian, Cherokee and Mtavruli (Java 8: unchanged), Latin Extended-D
     # (mapped up to U+A7AA, unchanged past it), Deseret, Osage (unchanged), "№"
     "Ἀ", "ἱ", "Ὠ", "ᾈ", "Ḃ", "ạ", "Ⅻ", "Ⓐ", "Ａ", "ｚ", "Ⰰ", "Ⲁ", "Ⴀ", "ა", "Ꭰ", "Ა", "Ꝁ", "Ꞓ", "Ꞡ", "Ꞵ",
     "\U00010400", "\U00010427", "\U00010428", "\U000104B0", "№", "ℤ", "ﬀ",
     # the 18 characters Java lower-cases by rule (İ → "i̇", Σ by Final_Sigma, length-changing capitals), Greek
     # letters around Σ, and case-ignorables its context skips (apostrophe, period, colon, middle dot, combining
     # acute, modifier letters, the SMP's mathematical capitals as cased letters)
     "İ", "Σ", "Σ", "Σ", "Ⱥ", "Ⱦ", "ẞ", "Ω", "K", "Å", "Ɫ", "Ɽ", "Ɑ", "Ɱ", "Ɐ", "Ɒ", "Ȿ", "Ɀ", "Ɥ", "Ɦ",
     "Α", "Ο", "Δ", "σ", "'", ".", ":", "·", "\u0301", "ʰ", "ᵃ", "\U0001D400"]
_SPACES = [" ", " ", " ", "\t", "\n", "\x0b", "\f", "\r"]


def random_texts(rng, n, max_len):
    out = []
    for _ in range(n):
        L = int(rng.integers(0, max_len + 1))
        chars = [(_SPACES[rng.integers(len(_SPACES))] if rng.random() < 0.18 else _ALPHABET[rng.integers(len(_ALPHABET))])
                 for _ in range(L)]
        out.append("".join(chars))
    return out


def test_known_answers_on_device(ctx, oracle):
    import stc

    texts = [t for t, _ in JAVA_SPLIT_KNOWN] + ["Hello  WORLD\tÄrger ÜBER Straße", "×ÞÀ"]
    got = stc.Tokenizer(ctx=ctx).transform(texts)
    assert got == [oracle.tokenize(t) for t in texts]
    for (_, exp), g in zip(JAVA_SPLIT_KNOWN, got):
        assert g == exp


@pytest.mark.parametrize("n,max_len", [(0, 0), (1, 0), (300, 12), (2000, 200), (40, 5000)])
def test_random_texts_bit_exact(ctx, oracle, n, max_len):
    import stc

    rng = np.random.default_rng(n * 7 + max_len)
    texts = random_texts(rng, n, max_len)
    texts += ["   ", "", "a" * 64, "b" * 65, " " * 64 + "x", "x" + " " * 130]  # chunk edges, all-space
    got = stc.Tokenizer(ctx=ctx).transform(texts)
    exp = [oracle.tokenize(t) for t in texts]
    assert len(got) == len(exp)
    for g, e, t in zip(got, exp, texts):
        assert g == e, repr(t)


@pytest.mark.parametrize("text", ["İstanbul", "ΣΟΦΙΑ", "ΟΔΟΣ", "ΟΔΟΣ ΟΔΟΣ. ΣΑΣ'Σ", "Σ", "ΑΣ", "ΣΑ", "Α.Σ.Β", "Α'Σ",
                                  "ΑΣ\u0301", "ΑΣ\u0301Β", "ΑΣ1", "ʰΣ", "\U0001D400Σ", "ΑΣ\U0001D400", "ΣΣΣ",
                                  "Ⱥx", "STRAẞE", "10 \u2126", "300 \u212a", "Ɫa", "Ɦb", "Å ⱥ ȿ",
                                  "İ" * 40, "Σ" * 33 + " ΑΣ", "x" * 63 + "İ" + "y", "x" * 62 + "ẞ" + "z" * 70])
def test_rule_cased_characters_bit_exact(ctx, oracle, text):
    """The 18 code points Java 8 lower-cases by rule (they were rejected through round 3):
    İ → "i̇" (2 → 3 bytes), Σ → ς / σ by its Final_Sigma context (case-ignorables skipped, word and string
    edges, a Σ straddling the 64-byte step), and the capitals whose lower case changes UTF-8 length
    (K → k shrinks 3 → 1).  Tokens are bit-exact against oracle.tokenize, also beside plain text."""
    import stc

    tok = stc.Tokenizer(ctx=ctx)
    texts = ["fine text", text, text.upper() + " " + text, ""]
    got = tok.transform(texts)
    assert got == [oracle.tokenize(t) for t in texts], repr(text)


def test_two_byte_scripts_lower_cased(ctx, oracle):
    """Cyrillic, Greek, Latin Extended-A/B and Armenian capitals follow Java 8's toLowerCase."""
    import stc

    texts = ["Москва ПРИВЕТ Ёлка", "ЇЖАК Ґанок", "ΑΘΗΝΑ Ωμέγα", "ĞÜZEL ŁÓDŹ ǄEMAL Ǆ", "ԱՐԱՐԱՏ",
             "Ϳ Ԩ Ԯ", "Źdźbło\tŻÓŁW"]
    got = stc.Tokenizer(ctx=ctx).transform(texts)
    assert got == [oracle.tokenize(t) for t in texts]
    assert got[0] == ["москва", "привет", "ёлка"] and got[2] == ["αθηνα", "ωμέγα"]
    assert got[5] == ["Ϳ", "Ԩ", "Ԯ"]  # assigned after Unicode 6.2: Java 8 leaves them as they are


def test_three_and_four_byte_scripts_lower_cased(ctx, oracle):
    """Past U+07FF: Greek Extended (Walden's γεἱβω), Latin Extended Additional, letterlike, enclosed and
    fullwidth capitals, Glagolitic, Coptic, Georgian, Deseret; "№" and CJK pass; the scripts Java 8 does
    not case (Cherokee, Mtavruli, Latin Extended-D past U+A7AA, Osage) stay as they are."""
    import stc

    texts = ["ἈΘΗΝΑΙ γεἱβω ὉΔΟΥ", "ḂḞḞ ẠẸỊ ỲỸ", "ⅫⅣ ⒶⒷ ＡＢＣ ｘｙｚ", "ⰀⰁ ⲀⲂ ႠႡ", "\U00010400\U00010410\U00010427 x",
             "Лицензия № 2", "ᎠᎡ ᲐᲑ ꞫꞲ \U000104B0", "漢字 😀 ℤ ﬀ"]
    got = stc.Tokenizer(ctx=ctx).transform(texts)
    assert got == [oracle.tokenize(t) for t in texts]
    assert got[0] == ["ἀθηναι", "γεἱβω", "ὁδου"] and got[5] == ["лицензия", "№", "2"]
    assert got[4][0] == "\U00010428\U00010438\U0001044f"
    assert got[6] == ["ᎠᎡ", "ᲐᲑ", "ꞫꞲ", "\U000104B0"]


def test_reference_books_bit_exact(ctx, oracle):
    """Text of the reference's own corpora (resources/books/<Lang>, tests/golden/books_text.json):
    Russian and Ukrainian (Cyrillic) and the five Latin-script languages, tokens bit-exact."""
    import stc
    from helpers import golden_json

    books = golden_json("books_text.json")
    texts = [s["text"] for lang in sorted(books) for s in books[lang]]
    assert any("\u0400" <= ch <= "\u04ff" for ch in "".join(texts))
    got = stc.Tokenizer(ctx=ctx).transform(texts)
    assert got == [oracle.tokenize(t) for t in texts]
    htf = stc.HashingTF(ctx=ctx)  # Spark 2.4.3's tail
    d = htf.transform_text_device(texts)
    try:
        m = d.download()
    finally:
        d.free()
    ip, ix, vv = oracle.hashing_tf([oracle.tokenize(t) for t in texts], 1 << 18, False, oracle.HASH_SPARK24)
    assert np.array_equal(m.indptr, ip) and np.array_equal(m.indices, ix) and np.array_equal(m.values, vv)


@pytest.mark.parametrize("binary", [False, True])
def test_fused_tokenize_hashing_tf(ctx, oracle, binary):
    import stc

    rng = np.random.default_rng(11)
    texts = random_texts(rng, 500, 300) + ["", "   ", "Über ÜBER über"]
    for algo, variant in (("murmur3", 0), ("murmur3-spark24", 1)):
        htf = stc.HashingTF(numFeatures=1 << 18, binary=binary, hashAlgorithm=algo, ctx=ctx)
        d = htf.transform_text_device(texts)
        try:
            got = d.download()
        finally:
            d.free()
        ip, ix, vv = oracle.hashing_tf([oracle.tokenize(t) for t in texts], 1 << 18, binary, variant)
        assert np.array_equal(got.indptr, ip)
        assert np.array_equal(got.indices, ix)
        assert np.array_equal(got.values, vv)
