"""stc — MI355X-native HashingTF → IDF → online-LDA hot path of borisfoko/Spark-Text-Clustering.

The compute lives in libstc.so (HIP kernels for gfx950 behind the C ABI in include/stc.h); this
package is the host-side mirror of the Spark ML interface the reference's pipeline uses.
"""
from ._lib import (STC_ERR_HIP, STC_ERR_INVALID_ARG, STC_ERR_OOM, STC_ERR_RCCL, STC_ERR_STATE, STC_F32, STC_F64, STC_MIXED,
                   STC_HASH_SPARK24, STC_HASH_STANDARD, STC_LAYOUT_KV, STC_LAYOUT_VK, StcError, StcIllegalArgument,
                   load)
from . import io
from .clustering import (LDA, ML_LDA_DEFAULT_SEED, DistributedLDAModel, LdaGroup, LdaHandle, LDAModel, MllibLDA,
                         OnlineLDAOptimizer, reference_mini_batch_fraction)
from .core import Context, CsrMatrix, DeviceCsr
from .feature import IDF, DeviceTokens, HashingTF, IDFModel, Tokenizer, encode_texts, encode_tokens

__all__ = [
    "Context", "CsrMatrix", "DeviceCsr", "HashingTF", "IDF", "IDFModel", "Tokenizer", "encode_texts", "encode_tokens", "LDA",
    "LDAModel", "DistributedLDAModel", "LdaGroup", "LdaHandle", "io", "MllibLDA", "OnlineLDAOptimizer", "ML_LDA_DEFAULT_SEED",
    "reference_mini_batch_fraction", "StcError", "StcIllegalArgument", "load", "STC_F32", "STC_F64", "STC_MIXED",
    "STC_HASH_STANDARD", "STC_HASH_SPARK24", "STC_LAYOUT_VK", "STC_LAYOUT_KV", "STC_ERR_INVALID_ARG", "STC_ERR_HIP",
    "STC_ERR_RCCL", "STC_ERR_OOM", "STC_ERR_STATE",
]
