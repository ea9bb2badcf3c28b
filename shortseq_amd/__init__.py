"""shortseq_amd — MI355X-native batch 2-bit DNA encode / decode / hamming / dedup-count engine.

Drop-in for the reference's Python API (shortseq/__init__.py:1-14): pack, from_str, from_bytes,
ShortSeq64 / ShortSeq192 / ShortSeqVar, ShortSeqCounter, read_and_count_fastq, get_domain_*,
MIN_/MAX_*_NT.  Batch GPU entry points live in shortseq_amd.batch (HIP kernels behind the C ABI in
include/shortseq_amd.h).
"""
__version__ = "0.1.0"
