"""shortseq.short_seq_var (reference short_seq_var.pyx): ShortSeqVar and its length domain."""
from shortseq_amd import ShortSeqVar, get_domain_var  # noqa: F401
