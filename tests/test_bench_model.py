"""bench.py's algorithmic work model (CPU): the MACs per sample it prices every roofline with, against the
layer sizes of the oracle's network spec (MLP.cs:64-86 / MLPcpp:131-154) and SURVEY.md §8(d)'s figures."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


@pytest.mark.parametrize("net", [
    dict(net_depth=8, net_width=256, net_depth_condition=1, net_width_condition=128, skip_layer=4,
         min_deg_point=0, max_deg_point=16, deg_view=4),
    dict(net_depth=4, net_width=128, net_depth_condition=1, net_width_condition=128, skip_layer=4,
         min_deg_point=0, max_deg_point=16, deg_view=4),
    dict(net_depth=5, net_width=96, net_depth_condition=3, net_width_condition=40, skip_layer=2,
         min_deg_point=2, max_deg_point=10, deg_view=2),
])
def test_net_macs_match_layer_sizes(oracle, net):
    import bench

    spec = oracle.Spec(D=net["net_depth"], W=net["net_width"], Dc=net["net_depth_condition"],
                       Wc=net["net_width_condition"], skip=net["skip_layer"], min_deg=net["min_deg_point"],
                       max_deg=net["max_deg_point"], deg_view=net["deg_view"])
    sizes = oracle.layer_sizes(spec)
    L = len(sizes) // 2
    fwd, dx, dw = bench.net_macs(net)
    assert fwd == dw == int(sum(sizes[:L]))  # every weight once forward, once in dW
    # dX: every weight row block that multiplies a hidden activation (not the IPE / view-PE columns)
    D, W, Dc, Wc = spec.D, spec.W, spec.Dc, spec.Wc
    assert dx == (D - 1) * W * W + W + Wc * W + (Dc - 1) * Wc * Wc + 3 * Wc


def test_reference_constants_and_survey_figures():
    import bench

    ref = dict(net_depth=8, net_width=256, net_depth_condition=1, net_width_condition=128, skip_layer=4,
               min_deg_point=0, max_deg_point=16, deg_view=4)
    assert bench.net_macs(ref) == (bench.MACS_FWD, bench.MACS_DX, bench.MACS_DW)
    assert 2 * sum(bench.net_macs(bench.CONFIG0_NET)) == 459264  # config 1, FLOP/sample
