"""Extract the stereo rectification calibration (LEFT/RIGHT K, D, R, P, size) and Camera.bf
from the reference's Examples/Stereo/EuRoC.yaml into tests/golden/euroc_stereo_calib.json
(data fixture: the GPU box has no /root/reference).  Run from the repo root."""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "orb-slam3-noted_amd"))
from slamhot.euroc import read_settings  # noqa: E402

s = read_settings("/root/reference/Examples/Stereo/EuRoC.yaml")
out = {k: (v.tolist() if hasattr(v, "tolist") else v) for k, v in s.items()
       if k.startswith(("LEFT.", "RIGHT.")) or k in ("Camera.fx", "Camera.fy", "Camera.cx", "Camera.cy", "Camera.bf",
                                                    "Camera.width", "Camera.height")}
(ROOT / "tests" / "golden" / "euroc_stereo_calib.json").write_text(json.dumps(out, indent=1))
print(sorted(out))
