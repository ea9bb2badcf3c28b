"""`shortseq` — the reference's import name for the shortseq_amd drop-in.

The reference's users and tests write `import shortseq as sq` and `from shortseq import ShortSeq64`
(shortseq/__init__.py:1-14, tests/unit_tests_main.py:6-9).  This package re-exports the shortseq_amd
drop-in under that name, with the reference's module layout (shortseq.short_seq, .short_seq_64,
.short_seq_192, .short_seq_var, .counter), so such code runs unchanged.  Nothing is implemented here.
"""
from shortseq_amd import (  # noqa: F401
    pack, from_str, from_bytes, from_words,
    ShortSeq64, ShortSeq192, ShortSeqVar, ShortSeqCounter, read_and_count_fastq,
    get_domain_64, get_domain_192, get_domain_var,
    MIN_VAR_NT, MAX_VAR_NT, MIN_192_NT, MAX_192_NT, MIN_64_NT, MAX_64_NT,
)
from shortseq_amd import __version__  # noqa: F401
