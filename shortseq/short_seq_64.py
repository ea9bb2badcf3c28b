"""shortseq.short_seq_64 (reference short_seq_64.pyx): ShortSeq64 and its length domain."""
from shortseq_amd import ShortSeq64, get_domain_64  # noqa: F401
