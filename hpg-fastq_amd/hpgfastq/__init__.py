"""hpgfastq — Python view of the libhpgq C-ABI (include/hpgq.h).

This is the ctypes binding a maintainer would add on the reference side
(INTEGRATION.md); tests/ and bench.py drive the HIP engine through it.  It
never computes anything itself: every call goes to libhpgq.so, and importing
fails loudly if the library has not been built (`make -C hpg-fastq_amd`).
"""
from ._abi import (  # noqa: F401
    LIB_PATH, lib, HpgqError, Params, Batch, Synth, Summary,
    NUM_SCALARS, S_NUM_INPUT, S_NUM_PASSED, S_NUM_FAILED, S_NUM_EDITED,
    S_NUM_STATS, S_ACC_MEANQ_FX16, S_LONG_READS, MEANQ_BINS, GC_BINS,
    NO_VALUE, MIN_VALUE, MAX_VALUE, LMAX_LIMIT, MAX_EDIT_LENGTH, DEVICE_SLACK, CGR_ALL_READS, CGR_ONLY_VALID_READS, CGR_PATH_AUTO, CGR_PATH_EXACT,
    counters_len, layout, check, params_default, exported_symbols,
)
from .engine import Engine, ChaosGame, Kmers, Parser, summary, complete_prefix  # noqa: F401
from .engine import (cgr_write_gs, cgr_load_gs, cgr_table_dif, cgr_dif_stats,  # noqa: F401
                     cgr_normalize_quality, cgr_write_pgm, cgr_write_images)
from .options import parse_range, filter_params, edit_params, stats_params  # noqa: F401
