"""Host option semantics (hpgfastq.options) vs the reference's rules:
parse_range src/commons_fastq.c:31-103, defaults src/filter_fastq.c:195-206,
filter_on src/stats_options.c:177-213, edit src/edit_fastq.c:148-171."""
import pytest

import hpgfastq as H
from hpgfastq.options import RangeError, filter_on

NV = H.NO_VALUE


@pytest.mark.parametrize("text,want", [
    ("20,40", (20, 40)), ("20,", (20, NV)), (",40", (NV, 40)), ("20", (20, NV)),
    ("0,0", (0, 0)), ("7,7", (7, 7)), ("12abc,30", (12, 30)), (None, (NV, NV)),
])
def test_parse_range_accepts(text, want):
    assert H.parse_range(text) == want


@pytest.mark.parametrize("text", ["40,20", "-5,10", "5,-10", "abc", ",x", "x,"])
def test_parse_range_rejects(text):
    with pytest.raises(RangeError):
        H.parse_range(text)


def test_stats_defaults_no_filter():
    p = H.stats_params(lmax=150)
    assert p.filter_on == 0 and p.stats_on == 1
    assert (p.min_read_length, p.max_read_length) == (H.MIN_VALUE, H.MAX_VALUE)
    assert (p.min_read_quality, p.max_read_quality) == (H.MIN_VALUE, H.MAX_VALUE)


def test_stats_c2_flags():
    p = H.stats_params(lmax=150, read_quality_range="20,", read_length_range="50,")
    assert p.filter_on == 1
    assert (p.min_read_quality, p.max_read_quality) == (20, H.MAX_VALUE)
    assert (p.min_read_length, p.max_read_length) == (50, H.MAX_VALUE)


@pytest.mark.parametrize("opts,on", [
    ({}, False),
    ({"read_length_range": "10,"}, True),
    ({"read_quality_range": "20,"}, True),
    ({"left_length": 5}, False),                      # length without a range
    ({"left_length": 5, "left_quality_range": "20,"}, True),
    ({"right_length": 5, "right_quality_range": "20,"}, True),
    ({"max_N": 0}, True),
    ({"max_out_of_quality": 3}, False),               # needs a quality range
    ({"max_out_of_quality": 3, "read_quality_range": "20,"}, True),
])
def test_filter_on_rules(opts, on):
    assert filter_on(opts) is on


def test_filter_requires_a_flag():
    with pytest.raises(RangeError):
        H.filter_params(lmax=150)
    p = H.filter_params(lmax=150, max_N=0)
    assert p.stats_on == 0 and p.filter_on == 1 and p.max_N == 0


def test_edit_moves_left_right_into_edit_fields():
    p = H.edit_params(lmax=150, left_length=10, left_quality_range="20,", right_length=30,
                      right_quality_range="15,")
    assert p.edit_on == 1 and p.filter_on == 0
    assert (p.edit_left_length, p.edit_min_left_quality) == (10, 20)
    assert (p.edit_right_length, p.edit_min_right_quality) == (30, 15)
    assert p.left_length == 0 and p.right_length == 0   # filter's windows forced off
    with pytest.raises(RangeError):
        H.edit_params(lmax=150, read_length_range="10,")   # nothing to edit
    with pytest.raises(RangeError):   # trims are two 16-bit fields
        H.edit_params(lmax=150, left_length=65536, left_quality_range="20,")
    assert H.edit_params(lmax=150, right_length=65535, right_quality_range="20,").edit_right_length == 65535


def test_quality_encoding():
    assert H.stats_params(quality_encoding="phred64").phred == 64
    with pytest.raises(RangeError):
        H.stats_params(quality_encoding="solexa")
