"""shortseq_amd — MI355X-native batch 2-bit DNA encode / decode / hamming / dedup-count engine.

Drop-in for the reference's Python API (shortseq/__init__.py:1-14): pack, from_str, from_bytes,
ShortSeq64 / ShortSeq192 / ShortSeqVar, ShortSeqCounter, read_and_count_fastq, get_domain_*,
MIN_/MAX_*_NT.  Batch GPU entry points live in shortseq_amd.batch (HIP kernels behind the C ABI in
include/shortseq_amd.h).
"""
try:
    from ._shortseq import (  # noqa: F401
        pack, from_str, from_bytes, from_words,
        ShortSeq64, ShortSeq192, ShortSeqVar, ShortSeqCounter, read_and_count_fastq,
        get_domain_64, get_domain_192, get_domain_var,
    )
except ImportError as e:  # dev checkout without the built extension: build it in-tree once
    if "_shortseq" not in str(e):
        raise
    from .build import build_cython as _bc
    _bc()
    from ._shortseq import (  # noqa: F401
        pack, from_str, from_bytes, from_words,
        ShortSeq64, ShortSeq192, ShortSeqVar, ShortSeqCounter, read_and_count_fastq,
        get_domain_64, get_domain_192, get_domain_var,
    )

MIN_VAR_NT, MAX_VAR_NT = get_domain_var()
MIN_192_NT, MAX_192_NT = get_domain_192()
MIN_64_NT, MAX_64_NT = get_domain_64()

__version__ = "0.1.0"
