"""The C-ABI library: loads without a GPU, exports every symbol include/slamhot.h declares,
and refuses to run without a gfx950 device (no CPU fallback)."""
import ctypes as C
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def declared_symbols():
    hdr = (ROOT / "include" / "slamhot.h").read_text()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(slamhot_\w+)\s*\(", hdr)))


def test_header_declares_api():
    syms = declared_symbols()
    for s in ("slamhot_extractor_create", "slamhot_extract", "slamhot_extract_batch_device",
              "slamhot_vocab_transform", "slamhot_search_by_bow"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    import slamhot
    lib = slamhot.lib()
    missing = [s for s in declared_symbols() if not hasattr(lib, s)]
    assert not missing, missing


def test_no_cpu_fallback_without_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import slamhot
    n = slamhot.device_count()
    assert n == 0
    with pytest.raises(slamhot.SlamError) as e:
        slamhot.ORBextractor()
    assert e.value.status == slamhot.SLAM_ENODEV
    with pytest.raises(slamhot.SlamError):
        slamhot.ORBmatcher()


def test_status_strings():
    import slamhot
    assert slamhot.status_string(0) == "ok"
    assert "gfx950" in slamhot.status_string(slamhot.SLAM_ENODEV)
