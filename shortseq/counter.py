"""shortseq.counter (reference counter.pyx:10-70): ShortSeqCounter and read_and_count_fastq."""
from shortseq_amd import ShortSeqCounter, read_and_count_fastq  # noqa: F401
