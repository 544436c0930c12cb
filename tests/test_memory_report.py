"""The harness memory report (zero_amd/training_utils/memory.py, the reference's
zero/training_utils/memory.py:37-50): torch's figures as the reference prints them, and — when
buffers are placed outside torch's allocator — the combined residency comparable to the
reference's."""
from zero_amd.training_utils.memory import MemoryReport


def test_report_adds_placed_buffers_to_a_combined_total():
    r = MemoryReport(10.0, 10.0, 40.0, 10.0, 10.0, 40.0, allocated_mb=100.0, max_allocated_mb=150.0,
                     placed_mb=2048.0, placed_peak_mb=4096.0)
    text = "\n".join(r.lines("After step", 0))
    assert "Total allocated: 100.00 MB" in text and "Max allocated: 150.00 MB" in text
    assert "Placed outside torch's allocator: 2048.00 MB" in text
    assert "Total incl. placed: 2148.00 MB (max <= 4246.00 MB" in text
    assert r.total_mb == 2148.0 and r.max_total_mb == 4246.0


def test_report_without_placed_buffers_is_the_reference_format():
    r = MemoryReport(1.0, 1.0, 2.0, 1.0, 1.0, 2.0, allocated_mb=5.0, max_allocated_mb=6.0)
    lines = r.lines("Before", 1)
    assert lines[0] == "\nGPU 1 - Before:" and len(lines) == 7  # the reference's five lines
    assert not any("placed" in ln for ln in lines)
