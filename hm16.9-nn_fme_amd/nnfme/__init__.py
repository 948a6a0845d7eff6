"""nnfme — MI355X-native fractional-pel motion estimation for HM-16.9-NN_FME.

Host side of the path above the C-ABI (include/fme.h): numpy mirrors of the job/result
structs (abi), per-QP NN weight sets (weights), synthetic YUV and job generators (synth),
the ctypes binding of libfme_amd.so (runtime) and frame sharding over RCCL (dist).
"""
from .abi import JOB_DTYPE, RESULT_DTYPE, JOB_EMI, JOB_BIPRED, JOB_LOSSLESS  # noqa: F401

__all__ = ["abi", "weights", "synth", "runtime", "dist"]
