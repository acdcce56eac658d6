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
