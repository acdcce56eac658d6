"""The launch's work plan (rt_dev_path.h start_item / fold_frame, rt_api.cpp
regions): every (frame, block) pair of the main part traced by exactly one
item, every slot written once and read by its own frame's collect in block
order -- with and without lead items (knob block_lead), over a sweep of
frame / block / region shapes (tools/plan_model.py restates the formulas)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tools"))
import plan_model  # noqa: E402


def test_plan_exact_cover():
    plan_model.main()


def test_headline_lead_slots():
    # the headline launch: 20 frames x 8 blocks, one tail pair, 18 whole
    # pixel-region frames; lead items of 4 blocks cut its block items 15 -> 7
    fp, fl, lead, nreg, c0 = plan_model.plan(20, 8, 144, 159, 4)
    assert (fp, fl, lead, nreg, c0) == (18, 20, 4, 7, 0)
    fp, fl, lead, nreg, c0 = plan_model.plan(20, 8, 144, 159, 0)
    assert (fp, fl, lead, nreg, c0) == (18, 18, 0, 15, 0)


def test_schedule_knob_test_shapes():
    # tests/test_gpu_parity.py test_schedule_knobs_identical: 72 x 40, 64 spp,
    # depth 10, 3 frames, one workgroup per CU (65,536 lanes). The default
    # tail takes every pair; the short tail leaves a main part whose regions
    # the block region picks.
    L = 65536
    assert plan_model.host_plan(2880, 64, 10, 3, L)["qmain"] == 0
    T = (0, 0, 0.01)
    p = plan_model.host_plan(2880, 64, 10, 3, L, tail=T, block_region=0.3)
    assert (p["fp"], p["fl"], p["lead"], p["c0"]) == (2, 3, 2, 0)
    p = plan_model.host_plan(2880, 64, 10, 3, L, tail=T, block_region=0.55, block_align=False,
                             block_lead=3)
    assert (p["fp"], p["fl"], p["lead"], p["c0"]) == (1, 3, 3, 1)
    # the 3-frame 1080p launch of test_full_1080p64_lead_items, and the headline
    p = plan_model.host_plan(1920 * 1080, 64, 16, 3, 262144)
    assert (p["fp"], p["fl"], p["lead"]) == (1, 3, 2)
    p = plan_model.host_plan(1920 * 1080, 64, 16, 20, 262144)
    assert (p["qpix"], p["fp"], p["fl"], p["lead"], p["nreg"]) == (144, 18, 20, 2, 11)
