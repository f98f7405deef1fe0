"""bench.py's roofline objects from a synthetic KernelTimer summary (CPU):
every fraction is a fraction of its peak, and the ROIAlign backward's counter
bytes (one PMC "launch" = the whole backward) are divided by the backward's
summed launch time, not by one launch's."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_kernel_report_fractions_and_roi_backward_accounting():
    import bench
    summary = {"conv2d_split": (10, 0.8, 10 * 11.7e9), "roi_align_bwd": (5, 0.255, 5.0e8)}
    extras = {"roi_align_bwd": {"unique_bytes": 2.7e7}}
    rep = bench.kernel_report(summary, mode="train", extras=extras)
    conv, roi = rep["conv2d_split"], rep["roi_align_bwd"]
    assert 0 < conv["frac"] < 1 and conv["unit"] == "TFLOP/s"
    assert roi["bytes_model"] == "unique" and 0 < roi["frac"] < 1
    if roi.get("traffic"):  # the committed PMC summary is present
        assert roi["traffic_per"].startswith("backward op")
        want = roi["traffic"] / 0.255e-3 / 1e9
        assert abs(roi["achieved_counter"] - want) < 0.2
        assert roi["frac_counter"] < 1
