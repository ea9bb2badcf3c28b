"""shortseq.short_seq (reference short_seq.pyx:13-36): the pack / from_str / from_bytes dispatch."""
from shortseq_amd import pack, from_str, from_bytes  # noqa: F401
