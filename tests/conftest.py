import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT / "orb-slam3-noted_amd", ROOT / "tests", ROOT):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")
    # torch's HIP runtime must come up before libslamhot's first device call in this process
    # (the device-resident tests hand torch allocations to the library)
    markexpr = getattr(config.option, "markexpr", "") or ""
    if "not gpu" not in markexpr:
        try:
            import torch
            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:
            pass


@pytest.fixture(scope="session")
def gpu_extractor_factory():
    import slamhot
    made = []

    def make(**kw):
        ex = slamhot.ORBextractor(**kw)
        made.append(ex)
        return ex

    yield make
    for ex in made:
        ex.close()
