"""tools/lds_bank_model.py: the LDS lane-group model behind the conv kernels' layouts
(cnn_fused.hip comments quote these factors; LDS cycles per conflict-free cycle)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))

import lds_bank_model as m  # noqa: E402


def test_lane_group_rules():
    # 64 lanes reading 16 consecutive bytes each: conflict-free ds_read_b128
    assert m.b128([16 * lane for lane in range(64)]) == 1.0
    # every lane of a 16-lane group on the same bank, distinct addresses: 16-way
    assert m.b128([256 * lane for lane in range(64)]) == 16.0
    # identical addresses broadcast
    assert m.b128([0] * 64) == 1.0
    assert m.tr16([8 * lane for lane in range(64)]) == 1.0


def test_shipped_layout_factors():
    none = lambda y, x: 0  # noqa: E731
    # conv3 backward: a2 in 12-wide rows makes the transposed reads conflict-free
    assert m.conv3_bwd_a2(m.swz(lambda y, x: y * 9 + x, 72, none))[0] == 2.0
    assert m.conv3_bwd_a2(m.swz(lambda y, x: y * 12 + x, 80, none))[0] == 1.0
    # da3 image: 72 -> 80-element rows, dgrad b128 reads 2.75 -> 2.0
    assert m.conv3_bwd_da3(m.swz(lambda y, x: y * 11 + x, 72, none))[:2] == (2.75, 2.0)
    assert m.conv3_bwd_da3(m.swz(lambda y, x: y * 11 + x, 80, none))[:2] == (2.0, 2.0)
    # conv2 backward da2 rows 72 -> 80: dgrad reads 2.71 -> 1.86
    assert m.conv2_bwd_da2(m.swz(lambda y, x: y * 12 + x, 72, none))[0] == 2.71
    assert m.conv2_bwd_da2(m.swz(lambda y, x: y * 12 + x, 80, none))[0] == 1.86
    # fused forward: frame rows of 28 positions make conv1's reads conflict-free
    assert m.conv_stack_fwd_conv1(80, 21) == 1.6
    assert m.conv_stack_fwd_conv1(80, 28) == 1.0


def test_forward_a1_a2_layout_factors():
    # conv2 of the fused forward: stride-2 reads of 40-element rows 2.0; a 9 x 10 grid over
    # phase images of 48-element rows 1.0 (40-element rows stay at 2.0)
    assert m.conv_stack_fwd_conv2(40, False) == 2.0
    assert m.conv_stack_fwd_conv2(40, True) == 2.0 and m.conv_stack_fwd_conv2(48, True) == 1.0
    # conv3: 49 pixels 1.75, a 7 x 9 grid (consecutive rows) 1.0
    assert m.conv_stack_fwd_conv3(80, False) == 1.75 and m.conv_stack_fwd_conv3(80, True) == 1.0


def test_conv2_backward_dgrad_grid():
    none = lambda y, x: 0  # noqa: E731
    # the 10 x 12 dgrad grid reads consecutive da2 rows: 1.86 -> 1.0 for 8 instead of 7 tiles
    assert m.conv2_bwd_da2(m.swz(lambda y, x: y * 12 + x, 80, none), grid12=True)[0] == 1.0
