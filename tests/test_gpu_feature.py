"""GPU parity: HashingTF (K1/K2, bit-exact) and IDF (K3–K5) through the C ABI vs the oracle and
the reference's own saved TF·IDF edges (tests/golden/{en,ge}_idf.npz)."""
import numpy as np
import pytest

from helpers import golden_npz, random_tokens

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("algo,variant", [("murmur3", 0), ("murmur3-spark24", 1)])
def test_hash_tokens_bit_exact(ctx, oracle, algo, variant):
    import stc

    rng = np.random.default_rng(1)
    docs = random_tokens(rng, 60)
    terms = [t for d in docs for t in d]
    for nf in (1 << 18, 1000, 7, 1 << 20):
        htf = stc.HashingTF(numFeatures=nf, hashAlgorithm=algo, ctx=ctx)
        got = htf.indices_of(terms)
        exp = [oracle.non_negative_mod(oracle.murmur3_x86_32(t.encode(), 42, variant), nf) for t in terms]
        assert np.array_equal(got, np.asarray(exp, np.int32)), nf


def test_murmur3_known_answers_on_device(ctx):
    """Public MurmurHash3_x86_32 vectors (seed 42 is Spark's; use numFeatures = 2^31 - 1 to read
    the non-negative residue of the signed hash)."""
    import stc

    from oracle import oracle as O

    htf = stc.HashingTF(numFeatures=(1 << 31) - 1, hashAlgorithm="murmur3", ctx=ctx)
    words = ["", "a", "ab", "abc", "abcd", "hello", "The quick brown fox jumps over the lazy dog"]
    got = htf.indices_of(words)
    for w, g in zip(words, got):
        assert g == O.non_negative_mod(O.murmur3_x86_32(w.encode(), 42), (1 << 31) - 1)


@pytest.mark.parametrize("binary", [False, True])
@pytest.mark.parametrize("algo,variant", [("murmur3", 0), ("murmur3-spark24", 1)])
def test_hashing_tf_csr_bit_exact(ctx, oracle, binary, algo, variant):
    import stc

    rng = np.random.default_rng(2)
    docs = random_tokens(rng, 300, max_len=80)
    docs[5] = []  # empty rows are kept (zero-length sparse vectors)
    docs[17] = ["same"] * 50
    for nf in (1 << 18, 97):
        out = stc.HashingTF(numFeatures=nf, binary=binary, hashAlgorithm=algo, ctx=ctx).transform(docs)
        ip, ix, vv = oracle.hashing_tf(docs, nf, binary, variant)
        assert np.array_equal(out.indptr, ip)
        assert np.array_equal(out.indices, ix)
        assert np.array_equal(out.values, vv)


def test_hashing_tf_all_empty(ctx):
    import stc

    out = stc.HashingTF(ctx=ctx).transform([[], [], []])
    assert out.shape == (3, 1 << 18) and out.nnz == 0


@pytest.mark.parametrize("tag", ["en", "ge"])
def test_idf_reference_edges_bit_exact(ctx, oracle, tag):
    """IDF(2).fit + the 1e-4 floor (LDAClustering.scala:177-188) reproduce every TF·IDF value the
    reference stored in its saved model, bit for bit."""
    import stc

    f = golden_npz(f"{tag}_idf.npz")
    V = int(f["vocab_size"])
    tf = stc.CsrMatrix(f["indptr"], f["indices"], f["tf"].astype(np.float64), V)
    model = stc.IDF(minDocFreq=int(f["min_doc_freq"]), ctx=ctx).fit(tf)
    assert model.numDocs == int(f["num_docs"])
    idf_o, df_o, m_o = oracle.idf_fit(tf.indptr, tf.indices, tf.values, V, int(f["min_doc_freq"]))
    assert np.array_equal(model.docFreq, df_o)
    assert np.max(np.abs(model.idf - idf_o) / np.maximum(np.abs(idf_o), 1e-300)) <= 1e-15
    out = model.transform(tf, zero_floor=1e-4)
    assert np.array_equal(out.indices, tf.indices)
    rel = np.abs(out.values - f["tfidf"]) / f["tfidf"]
    # device log() vs the JVM's: at most an ulp apart; north star asks for 1e-6 relative
    assert rel.max() <= 1e-15, rel.max()
    print(f"{tag}: {np.mean(out.values == f['tfidf']):.6f} of the stored edges reproduced bit for bit")


def test_idf_min_doc_freq_and_stock_transform(ctx, oracle):
    import stc

    rng = np.random.default_rng(3)
    V = 50
    rows = []
    for _ in range(40):
        ids = np.sort(rng.choice(V, size=int(rng.integers(0, 12)), replace=False))
        vals = rng.integers(0, 4, ids.size).astype(np.float64)  # explicit zeros don't count
        rows.append((ids, vals))
    tf = stc.CsrMatrix.from_rows(rows, V)
    for mdf in (0, 1, 3, 10):
        m = stc.IDF(minDocFreq=mdf, ctx=ctx).fit(tf)
        idf_o, df_o, _ = oracle.idf_fit(tf.indptr, tf.indices, tf.values, V, mdf)
        assert np.array_equal(m.docFreq, df_o)
        np.testing.assert_allclose(m.idf, idf_o, rtol=1e-15, atol=0)
        out = m.transform(tf)
        np.testing.assert_allclose(out.values, oracle.idf_transform(tf.indices, tf.values, idf_o),
                                   rtol=1e-15, atol=0)


def test_pipeline_hashing_idf_device_resident(ctx, oracle):
    """HashingTF → IDF with the TF matrix left in HBM (no host round trip between stages)."""
    import stc

    rng = np.random.default_rng(4)
    docs = random_tokens(rng, 200, max_len=60)
    htf = stc.HashingTF(numFeatures=1 << 12, ctx=ctx)  # default: Spark 2.4.3's legacy tail
    d = htf.transform_device(docs)
    model = stc.IDF(minDocFreq=2, ctx=ctx).fit_device(d)  # stays on the device (stc_idf_fit_dev)
    model.transform_device(d, zero_floor=1e-4)
    got = d.download()
    ip, ix, vv = oracle.hashing_tf(docs, 1 << 12, variant=oracle.HASH_SPARK24)
    idf_o, df_o, m_o = oracle.idf_fit(ip, ix, vv, 1 << 12, 2)
    assert np.array_equal(got.indices, ix)
    np.testing.assert_allclose(got.values, oracle.idf_transform(ix, vv, idf_o, floor=1e-4), rtol=1e-15, atol=0)
    # the device model's copy-out equals the host fit of the same matrix
    host = stc.IDF(minDocFreq=2, ctx=ctx).fit(stc.CsrMatrix(ip, ix, vv, 1 << 12))
    assert np.array_equal(model.idf, host.idf) and np.array_equal(model.docFreq, host.docFreq)
    assert model.numDocs == host.numDocs == m_o and np.array_equal(model.docFreq, df_o)
    model.free()
    assert np.array_equal(model.idf, host.idf)  # host arrays survive the device copy


def test_device_resident_tokens_synthetic_dictionary(ctx, oracle):
    """stc_tokens_upload + stc_hashing_tf_tokens (the featurisation bench's path) on the bench's own
    synthetic token generator (every UTF-8 tail length) vs the oracle, bit-exact."""
    import stc
    from stc import synth

    (blob, tok_off, doc_off), _ = synth.token_corpus(300, 40, n_words=5000, seed=9)
    dt = stc.DeviceTokens(ctx, blob, tok_off, doc_off)
    d = stc.HashingTF(numFeatures=1 << 18, ctx=ctx).transform_tokens_device(dt)
    got = d.download()
    d.free()
    dt.free()
    raw = blob.tobytes()
    docs = [[raw[tok_off[t]:tok_off[t + 1]] for t in range(doc_off[i], doc_off[i + 1])] for i in range(300)]
    ip, ix, vv = oracle.hashing_tf(docs, 1 << 18, False, oracle.HASH_SPARK24)
    assert np.array_equal(got.indptr, ip) and np.array_equal(got.indices, ix) and np.array_equal(got.values, vv)


@pytest.mark.parametrize("nf", [1 << 18, 97])
def test_hashing_tf_document_lengths(ctx, oracle, nf):
    """Every per-document sort path of K2 (hashing_tf.hip): register bitonic sorts of 1/2/4/8/16 keys
    per lane at both sides of each size boundary, the segmented radix sort past 1024 tokens, a long
    document of one repeated token, and runs that cross 64-key emit chunks."""
    import stc

    rng = np.random.default_rng(21)
    lens = [0, 1, 2, 63, 64, 65, 127, 128, 129, 255, 256, 257, 511, 512, 513, 1023, 1024, 1025, 3000, 20000]
    vocab = [f"w{i}" for i in range(5000)]
    docs = [[vocab[j] for j in rng.zipf(1.3, n) % len(vocab)] for n in lens]
    docs.append(["same"] * 2000)
    docs.append(["a", "b"] * 700)
    rng.shuffle(docs)
    out = stc.HashingTF(numFeatures=nf, ctx=ctx).transform(docs)
    ip, ix, vv = oracle.hashing_tf(docs, nf, False, oracle.HASH_SPARK24)
    assert np.array_equal(out.indptr, ip)
    assert np.array_equal(out.indices, ix)
    assert np.array_equal(out.values, vv)


@pytest.mark.parametrize("V", [1 << 18, 1 << 20, 1 << 21])
def test_idf_doc_freq_zipf_hot_ids(ctx, V):
    """doc_freq: heavy-hitter document frequencies on a Zipf corpus (hot ids in every row, more
    distinct ids per workgroup slice than LDS slots) equal the exact column counts of positive values;
    2^18 buckets take the LDS vocabulary tiles, 2^20 and 2^21 the radix-sorted runs."""
    import stc
    from stc import synth

    corpus = synth.zipf_corpus(40000 if V <= 1 << 18 else 5000, 200, V, seed=3)
    vals = corpus.values.copy()
    vals[::7] = 0.0  # explicit zeros do not count
    tf = stc.CsrMatrix(corpus.indptr, corpus.indices, vals, corpus.num_cols)
    m = stc.IDF(minDocFreq=0, ctx=ctx).fit(tf)
    df = np.bincount(tf.indices[vals > 0], minlength=tf.num_cols)
    assert np.array_equal(m.docFreq, df)
    assert m.numDocs == tf.num_rows


@pytest.mark.parametrize("V", [1000, (1 << 15) + 3, 1 << 18])
@pytest.mark.parametrize("D", [3, 7001])
def test_idf_doc_freq_tiled_and_binned(ctx, monkeypatch, V, D):
    """doc_freq's two LDS-tile counts (idf.hip: k_df_tiled, the default, one XCD's workgroups sharing a
    chunk group's index stream; k_df_bin + k_df_binned under STC_DF_BINNED=1) and HashingTF's single
    look-back pass vs its sorted-key passes (STC_TF_MODE=0, same CSR), and the transform with the
    model's hot-idf LDS table (default) and without it (STC_IDF_NO_CACHE=1) on a device-resident
    HashingTF matrix (values known positive: indices only) and on an uploaded matrix with explicit zeros
    (values read): exact column counts, with group counts that do and do not fill the XCD mapping."""
    import stc
    from stc import synth

    monkeypatch.setenv("STC_DF_BINNED", "1")
    monkeypatch.setenv("STC_TF_MODE", "0")
    monkeypatch.setenv("STC_IDF_NO_CACHE", "1")
    ctx_b = stc.Context(ctx.device)  # reads the knobs at stc_init
    for k in ("STC_DF_BINNED", "STC_TF_MODE", "STC_IDF_NO_CACHE"):
        monkeypatch.delenv(k)
    (blob, tok_off, doc_off), _ = synth.token_corpus(D, 150, n_words=40000, seed=11)
    csr = []
    for c in (ctx, ctx_b):
        dt = stc.DeviceTokens(c, blob, tok_off, doc_off)
        d = stc.HashingTF(numFeatures=V, ctx=c).transform_tokens_device(dt)
        host = d.download()
        csr.append(host)
        m = stc.IDF(minDocFreq=0, ctx=c).fit_device(d)
        assert np.array_equal(m.docFreq, np.bincount(host.indices, minlength=V))
        # the transform through the model's hot-idf LDS table (tag hits and misses) == host idf gathers
        m.transform_device(d, zero_floor=1e-4)
        w = np.where(m.idf == 0.0, 1e-4, m.idf)
        np.testing.assert_array_equal(d.download().values, host.values * w[host.indices])
        vals = host.values.copy()
        vals[::5] = 0.0  # explicit zeros do not count
        m2 = stc.IDF(minDocFreq=0, ctx=c).fit(stc.CsrMatrix(host.indptr, host.indices, vals, V))
        assert np.array_equal(m2.docFreq, np.bincount(host.indices[vals > 0], minlength=V))
        m.free()
        d.free()
        dt.free()
    ctx_b.close()
    # HashingTF's single look-back pass (default) and the round-3 passes give the same CSR
    a, b = csr
    assert np.array_equal(a.indptr, b.indptr) and np.array_equal(a.indices, b.indices)
    assert np.array_equal(a.values, b.values)


@pytest.mark.parametrize("algo,variant", [("murmur3", 0), ("murmur3-spark24", 1)])
def test_hash_window_lengths_and_alignments(ctx, oracle, algo, variant):
    """The 32-byte hash window (hashing_tf.hip load_win / murmur3_win): every token length 0–70 characters (1–2 UTF-8 bytes each)
    (inside the window, at its edge and past it) at every start alignment, in documents the fused
    hash + sort pass takes (≤ 256 tokens) and through stc_hash_tokens; the last token ends the blob."""
    import stc

    rng = np.random.default_rng(12)
    docs = []
    for pre in range(4):  # shifts every later token's start by pre bytes
        doc = ["p" * pre] if pre else []
        for n in range(71):
            doc.append(bytes(rng.integers(1, 256, n, dtype=np.uint8)).decode("latin-1"))
        docs.append(doc)
    htf = stc.HashingTF(numFeatures=1 << 18, hashAlgorithm=algo, ctx=ctx)
    out = htf.transform(docs)
    ip, ix, vv = oracle.hashing_tf(docs, 1 << 18, False, variant)
    assert np.array_equal(out.indptr, ip) and np.array_equal(out.indices, ix) and np.array_equal(out.values, vv)
    terms = [t for d in docs for t in d]
    got = htf.indices_of(terms)
    exp = [oracle.non_negative_mod(oracle.murmur3_x86_32(t.encode(), 42, variant), 1 << 18) for t in terms]
    assert np.array_equal(got, np.asarray(exp, np.int32))


def test_hashing_tf_single_pass_orders_and_fallback(ctx, monkeypatch):
    """HashingTF's look-back single pass (hashing_tf.hip single_pass; default), with the flat hash first
    (STC_TF_MODE=2), and with every look-back
    giving up at once (STC_TF_FAULT=1: the call falls back to the sorted-key passes and still succeeds):
    the same CSR as the sorted-key passes (STC_TF_MODE=0), bit for bit."""
    import stc
    from stc import synth

    (blob, tok_off, doc_off), _ = synth.token_corpus(3001, 120, n_words=30000, seed=21)
    got = {}
    for tag, env in [("single", {}), ("flat", {"STC_TF_MODE": "2"}),
                     ("fault", {"STC_TF_FAULT": "1"}), ("passes", {"STC_TF_MODE": "0"})]:
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        c = stc.Context(ctx.device)
        for k in env:
            monkeypatch.delenv(k)
        dt = stc.DeviceTokens(c, blob, tok_off, doc_off)
        d = stc.HashingTF(numFeatures=1 << 18, ctx=c).transform_tokens_device(dt)
        got[tag] = d.download()
        d.free()
        dt.free()
        c.close()
    ref = got.pop("passes")
    for tag, m in got.items():
        assert np.array_equal(m.indptr, ref.indptr), tag
        assert np.array_equal(m.indices, ref.indices), tag
        assert np.array_equal(m.values, ref.values), tag


def test_recycled_output_buffers_carry_no_stale_data(ctx, oracle):
    """A freed stc_dcsr / stc_didf hands its allocations back to the context (api.hip Recycler); the next
    HashingTF / IDF outputs of similar size reuse them: results of a large corpus, then a smaller one,
    then the large one again, each equal to the oracle (no entry of an earlier output survives)."""
    import stc
    from stc import synth

    big = synth.token_corpus(6000, 60, n_words=20000, seed=31)[0]
    small = synth.token_corpus(4500, 60, n_words=20000, seed=32)[0]
    for blob, tok_off, doc_off in (big, small, big):
        dt = stc.DeviceTokens(ctx, blob, tok_off, doc_off)
        d = stc.HashingTF(numFeatures=1 << 18, ctx=ctx).transform_tokens_device(dt)
        m = stc.IDF(minDocFreq=2, ctx=ctx).fit_device(d)
        m.transform_device(d, zero_floor=1e-4)
        got = d.download()
        raw = blob.tobytes()
        n_docs = doc_off.size - 1
        docs = [[raw[tok_off[t]:tok_off[t + 1]] for t in range(doc_off[i], doc_off[i + 1])] for i in range(n_docs)]
        ip, ix, vv = oracle.hashing_tf(docs, 1 << 18, False, oracle.HASH_SPARK24)
        idf_o, df_o, _ = oracle.idf_fit(ip, ix, vv, 1 << 18, 2)
        assert np.array_equal(got.indptr, ip) and np.array_equal(got.indices, ix)
        np.testing.assert_allclose(got.values, oracle.idf_transform(ix, vv, idf_o, floor=1e-4), rtol=1e-15, atol=0)
        assert np.array_equal(m.docFreq, df_o)
        m.free()
        d.free()
        dt.free()
