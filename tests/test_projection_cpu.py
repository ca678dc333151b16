"""tools/parts_projection.py --movers: the per-mover model of one
iteration of a row-partition part.  Sanity of the model itself on fixed kernel times (no GPU): the
orderings that follow from its assumptions must hold, and the numbers DESIGN.md quotes must come
out of the committed round-6 trace."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import parts_projection as pp  # noqa: E402

K = {"k_spmv_hot": 0.383, "k_seg_reduce": 0.006, "k_epilogue_grp": 0.100, "k_finalize": 0.006}
PASS = sum(K.values())


@pytest.mark.parametrize("P,mb", [(2, 87.0), (4, 101.0), (8, 89.0)])
def test_mover_model_orderings(P, mb):
    nc = 8 if P <= 4 else 4
    t = {name: pp.mover_ms(K, nc, mb, P, mv, early, chunked, r) for name, mv, early, chunked, r in pp.MOVERS}
    # nothing is faster than the pass alone, and nothing hides more than the whole transfer
    for name, v in t.items():
        assert v >= PASS - 1e-12, name
    ce_rate = min(pp.CE_STREAM_GBS * (P - 1), pp.CE_AGG_GBS)
    assert t["CE whole"] == pytest.approx(PASS + mb / ce_rate)
    assert t["link whole"] == pytest.approx(PASS + mb / (pp.LINK_GBS * (P - 1)))
    # chunking lets the copy engines run under the hot phases; whole runs cannot
    assert t["CE chunked"] < t["CE whole"]
    # a reserve slows every hot phase by 32 / (32 - r)
    assert t["link chunked early r2"] >= PASS + K["k_spmv_hot"] * (32 / 30 - 1) - 1e-12


def test_round6_p8_trace_projects_the_documented_speedups():
    """DESIGN.md §6 quotes 5.27x / 5.74x for the chunked copy-engine modes at P = 8 with this round's
    parts (profiles/r06/parts/)."""
    path = os.path.join(ROOT, "profiles", "r06", "parts", "kernel_trace_s26_p8_order_auto_staged_pack.csv")
    if not os.path.exists(path):
        pytest.skip("round-6 part trace not present")
    k = pp.part_kernels_ms(path)
    mb = 11084558 * 8 / 1e6
    ce_chunked = pp.mover_ms(k, 4, mb, 8, "ce", False, True)
    ce_early = pp.mover_ms(k, 4, mb, 8, "ce", True, True)
    assert round(3.095 / ce_chunked, 2) == 5.27
    assert round(3.095 / ce_early, 2) == 5.74
    assert max(pp.part_pass_us(path).values()) == pytest.approx(0.495, abs=5e-4)
