"""Option semantics of the hpg-fastq subcommands, mirrored for the host side.

parse_range follows src/commons_fastq.c:31-103; the defaulting and
`filter_on` rules follow src/stats_options.c:166-213,
src/filter_fastq.c:195-206 and src/edit_fastq.c:148-171.  The C++ CLI
(hpg-fastq_amd/host) implements the same rules; these Python twins let the
tests exercise them without a GPU.
"""
from ._abi import NO_VALUE, MIN_VALUE, MAX_VALUE, MAX_EDIT_LENGTH, params_default


class RangeError(ValueError):
    pass


def parse_range(text, what="range"):
    """'a,b' | 'a,' | ',b' | 'a' -> (min, max) with NO_VALUE for an open end."""
    if text is None:
        return NO_VALUE, NO_VALUE

    def _int(s, which):
        s = s.strip()
        # sscanf("%d") accepts a leading integer prefix
        i = 0
        if i < len(s) and s[i] in "+-":
            i += 1
        j = i
        while j < len(s) and s[j].isdigit():
            j += 1
        if j == i:
            raise RangeError(f"Invalid {which} value in the {what} ({text})")
        return int(s[:j])

    if "," in text:
        lo_s, hi_s = text.split(",", 1)
        hi = NO_VALUE if hi_s == "" else _int(hi_s, "maximum")
        lo = NO_VALUE if lo_s == "" else _int(lo_s, "minimum")
    else:
        lo, hi = _int(text, "minimum"), NO_VALUE
    if lo != NO_VALUE and lo < 0:
        raise RangeError(f"Invalid {what} ({text}). Minimum value ({lo}) must be greater than 0")
    if hi != NO_VALUE and hi < 0:
        raise RangeError(f"Invalid {what} ({text}). Maximum value ({hi}) must be greater than 0")
    if lo != NO_VALUE and hi != NO_VALUE and lo > hi:
        raise RangeError(f"Invalid {what} ({text}). Maximum value ({hi}) must be greater "
                         f"than minimum value ({lo})")
    return lo, hi


def _dflt(v, d):
    return d if v == NO_VALUE else v


def _filter_fields(o):
    """NO_VALUE -> MIN/MAX_VALUE, src/filter_fastq.c:195-206."""
    lmin, lmax_ = parse_range(o.get("read_length_range"), "read length range")
    qmin, qmax = parse_range(o.get("read_quality_range"), "read quality range")
    lqmin, lqmax = parse_range(o.get("left_quality_range"), "left quality range")
    rqmin, rqmax = parse_range(o.get("right_quality_range"), "right quality range")
    return dict(
        min_read_length=_dflt(lmin, MIN_VALUE), max_read_length=_dflt(lmax_, MAX_VALUE),
        min_read_quality=_dflt(qmin, MIN_VALUE), max_read_quality=_dflt(qmax, MAX_VALUE),
        max_out_of_quality=_dflt(o.get("max_out_of_quality", NO_VALUE), MAX_VALUE),
        left_length=_dflt(o.get("left_length", NO_VALUE), MIN_VALUE),
        min_left_quality=_dflt(lqmin, MIN_VALUE), max_left_quality=_dflt(lqmax, MAX_VALUE),
        right_length=_dflt(o.get("right_length", NO_VALUE), MIN_VALUE),
        min_right_quality=_dflt(rqmin, MIN_VALUE), max_right_quality=_dflt(rqmax, MAX_VALUE),
        max_N=_dflt(o.get("max_N", NO_VALUE), MAX_VALUE),
    )


def filter_on(o):
    """Any filter flag present (src/stats_options.c:177-213)."""
    n = 0
    n += o.get("read_length_range") is not None
    n += o.get("read_quality_range") is not None
    n += o.get("left_length", NO_VALUE) != NO_VALUE and o.get("left_quality_range") is not None
    n += o.get("right_length", NO_VALUE) != NO_VALUE and o.get("right_quality_range") is not None
    n += o.get("max_N", NO_VALUE) != NO_VALUE
    n += (o.get("max_out_of_quality", NO_VALUE) != NO_VALUE
          and o.get("read_quality_range") is not None)
    return n > 0


def _phred(o):
    enc = o.get("quality_encoding")
    if enc in (None, "phred33"):
        return 33
    if enc == "phred64":
        return 64
    raise RangeError(f"Invalid quality encoding value ({enc}). Valid values: phred33, phred64")


def stats_params(lmax=256, **o):
    """`hpg-fastq stats`: filter (if any flag) then stats on passed reads."""
    f = _filter_fields(o)
    return params_default(lmax=lmax, phred=_phred(o), stats_on=1,
                          filter_on=int(filter_on(o)), **f)


def filter_params(lmax=256, **o):
    """`hpg-fastq filter`: mask only (src/filter_fastq.c:134-155)."""
    if not filter_on(o):
        raise RangeError("Nothing to filter, no filter options specified !")
    f = _filter_fields(o)
    return params_default(lmax=lmax, phred=_phred(o), stats_on=0, filter_on=1, **f)


def edit_params(lmax=256, stats=False, **o):
    """`hpg-fastq edit`: trim, then filter with left/right forced off
    (src/edit_fastq.c:148-171)."""
    if not ((o.get("left_length", NO_VALUE) != NO_VALUE and o.get("left_quality_range"))
            or (o.get("right_length", NO_VALUE) != NO_VALUE and o.get("right_quality_range"))):
        raise RangeError("Nothing to edit, no edit options specified !")   # edit_options.c:228-231
    f = _filter_fields(o)
    # edit's filter_on ignores left/right (src/edit_options.c:190-215)
    fon = filter_on({k: v for k, v in o.items()
                     if k not in ("left_length", "left_quality_range",
                                  "right_length", "right_quality_range")})
    if max(f["left_length"], f["right_length"]) > MAX_EDIT_LENGTH:   # trims: two 16-bit fields
        raise RangeError(f"--left-length and --right-length must be at most {MAX_EDIT_LENGTH}")
    e = dict(edit_left_length=f["left_length"], edit_min_left_quality=f["min_left_quality"],
             edit_max_left_quality=f["max_left_quality"],
             edit_right_length=f["right_length"], edit_min_right_quality=f["min_right_quality"],
             edit_max_right_quality=f["max_right_quality"])
    f.update(left_length=MIN_VALUE, min_left_quality=MIN_VALUE, max_left_quality=MAX_VALUE,
             right_length=MIN_VALUE, min_right_quality=MIN_VALUE, max_right_quality=MAX_VALUE)
    return params_default(lmax=lmax, phred=_phred(o), stats_on=int(stats), filter_on=int(fon),
                          edit_on=1, **f, **e)
