"""Register allocation guard (CPU suite): the trace_samples instances of the built
librtamd.so must not spill more than the committed table says.

Spill counts, not instruction counts, decided most of round 2's wins and losses
(DESIGN.md §4): a compiler bump or an unrelated edit can push the sample-loop state of
an instance into scratch and cost 5-10% without changing a single result bit. This reads
the gfx950 code objects' metadata notes (tools/kernel_resources.py: VGPR / SGPR counts,
VGPR and SGPR spill counts, scratch bytes per lane) and compares every instance with
tests/golden/kernel_resources.json. A change that lowers a count passes (regenerate the
table with `python3 tools/kernel_resources.py --json > tests/golden/kernel_resources.json`
to pin the gain); one that raises a count fails here, before any GPU time is spent."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import kernel_resources as kr  # noqa: E402

TABLE = os.path.join(ROOT, "tests", "golden", "kernel_resources.json")
GUARDED = ("vgpr_spill_count", "sgpr_spill_count", "private_segment_fixed_size")


@pytest.fixture(scope="module")
def built():
    assert os.path.exists(kr.DEFAULT_LIB), "librtamd.so is not built (run __graft_entry__.build())"
    return {kr.readable(k): v for k, v in kr.kernel_resources(kr.DEFAULT_LIB).items() if "trace_samples" in k}


def test_every_instance_is_in_the_table(built):
    table = json.load(open(TABLE))
    assert set(built) == set(table), (sorted(set(built) - set(table)), sorted(set(table) - set(built)))


@pytest.mark.parametrize("inst", sorted(json.load(open(TABLE))))
def test_instance_spills_no_more_than_the_table(built, inst):
    want = json.load(open(TABLE))[inst]
    got = built[inst]
    worse = {k: (got[k], want[k]) for k in GUARDED if got[k] > want[k]}
    assert not worse, f"{inst}: {worse} (got, table)"
    # the occupancy the launch assumes: 3-wave instances <= 168 VGPRs, 4-wave <= 128
    waves = int(inst.split(",")[1])
    assert got["vgpr_count"] <= 512 // waves // 8 * 8


def test_metadata_decoder_reads_every_kernel_of_the_library():
    res = kr.kernel_resources(kr.DEFAULT_LIB)
    names = " ".join(v["name"] or "" for v in res.values())
    for k in ("resolve_samples", "numeric_eval", "kat_eval", "shard_pack", "shard_unpack", "quantise_lines"):
        assert k in names, k
