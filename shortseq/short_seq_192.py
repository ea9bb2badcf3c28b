"""shortseq.short_seq_192 (reference short_seq_192.pyx): ShortSeq192 and its length domain."""
from shortseq_amd import ShortSeq192, get_domain_192  # noqa: F401
