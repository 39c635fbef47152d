"""CPU: the C-ABI library loads and exports every symbol include/stc.h declares; host-side logic
(CSR containers, token encoding, Spark parameter validation) works without a GPU; the product
path fails loudly when no GPU is present."""
import ctypes
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_symbols():
    txt = open(os.path.join(ROOT, "include", "stc.h")).read()
    return sorted(set(re.findall(r"^\s*(?:const char\*|int|void)\s+(stc_\w+)\s*\(", txt, re.M)))


def test_header_declares_the_boundary():
    syms = _declared_symbols()
    for s in ("stc_hashing_tf", "stc_idf_fit", "stc_idf_transform", "stc_lda_create", "stc_lda_step",
              "stc_lda_next", "stc_lda_bound", "stc_lda_describe", "stc_lda_topic_distribution",
              "stc_comm_init", "stc_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    import stc

    lib = stc.load()
    missing = [s for s in _declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing
    from stc import _lib

    assert set(_lib.SIGNATURES) == set(_declared_symbols())
    assert lib.stc_abi_version() == 2


def test_library_is_gfx950_code():
    from stc import _lib

    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_fails_loudly_without_gpu():
    import stc

    # probe whatever devices this process can see (a GPU box may set HIP_VISIBLE_DEVICES to a real
    # device list): the test is about the no-GPU case only
    try:
        n = stc.Context.device_count()
    except stc.StcError:
        n = 0
    if n > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(stc.StcError):
        stc.Context(0)


def test_config_default_matches_spark_ml():
    import stc
    from stc import _lib

    cfg = _lib.LdaConfig()
    stc.load().stc_lda_config_default(ctypes.byref(cfg))
    assert cfg.k == 10 and cfg.vocab_size == 1 << 18
    assert cfg.tau0 == 1024.0 and cfg.kappa == 0.51 and cfg.mini_batch_fraction == 0.05
    assert cfg.gamma_shape == 100.0 and cfg.optimize_doc_concentration == 1
    assert cfg.topic_concentration == -1.0 and cfg.dtype == stc.STC_F64


def test_csr_container_and_rows():
    import stc

    m = stc.CsrMatrix.from_rows([([1, 5], [2.0, 1.0]), ([], []), ([0], [3.0])], 8)
    assert m.shape == (3, 8) and m.nnz == 3
    sub = m.rows([2, 0, 0])
    assert sub.indptr.tolist() == [0, 1, 3, 5]
    assert sub.indices.tolist() == [0, 1, 5, 1, 5]
    with pytest.raises(ValueError):
        stc.CsrMatrix([1, 2], [0], [1.0], 4)


def test_encode_tokens_utf8():
    import stc

    blob, tok, doc = stc.encode_tokens([["ab", "ж"], [], ["🙂"]])
    assert bytes(blob) == "abж🙂".encode()
    assert tok.tolist() == [0, 2, 4, 8] and doc.tolist() == [0, 2, 2, 3]


def test_spark_parameter_validation():
    import stc

    with pytest.raises(ValueError):
        stc.LDA(k=1)
    with pytest.raises(ValueError):
        stc.LDA(subsamplingRate=0.0)
    with pytest.raises(ValueError):
        stc.LDA(optimizer="em")
    with pytest.raises(ValueError):
        stc.LDA(learningOffset=0)
    with pytest.raises(ValueError):
        stc.HashingTF(numFeatures=0)
    with pytest.raises(ValueError):
        stc.IDF(minDocFreq=-1)
    with pytest.raises(ValueError):
        stc.OnlineLDAOptimizer().setMiniBatchFraction(1.5)
    with pytest.raises(ValueError):
        stc.MllibLDA().setOptimizer("gibbs")
    lda = stc.LDA()
    assert (lda.k, lda.maxIter, lda.learningOffset, lda.learningDecay, lda.subsamplingRate) == \
        (10, 20, 1024.0, 0.51, 0.05)
    assert lda.optimizeDocConcentration and lda.seed == stc.ML_LDA_DEFAULT_SEED


def test_reference_mini_batch_fraction():
    import stc

    assert stc.reference_mini_batch_fraction(51) == pytest.approx(0.05 + 1 / 51)
