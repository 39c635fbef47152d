"""GPU parity: the Tokenizer kernel K0 ([U] ml.feature.Tokenizer, toLowerCase.split("\\s")) through
the C ABI vs the oracle, bit-exact on tokens; Tokenizer → HashingTF fused on device vs oracle
tokenize + hashing_tf."""
import numpy as np
import pytest

from test_tokenizer_oracle import JAVA_SPLIT_KNOWN

pytestmark = pytest.mark.gpu

_ALPHABET = list("abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789.,;'\"-") + \
    ["Ä", "Ö", "Ü", "ß", "é", "È", "Ç", "×", "Þ", "µ", "\u00a0", "—", "“", "”", "€", "漢", "字", "😀"]
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


def test_unsupported_case_mapping_fails_loudly(ctx):
    import stc

    tok = stc.Tokenizer(ctx=ctx)
    for bad in ["İstanbul", "ĞÜZEL", "Ωmega", "Москва", "ＡＢＣ"]:
        with pytest.raises(ValueError, match="Tokenizer"):
            tok.transform(["fine text", bad])


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
