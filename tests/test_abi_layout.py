"""The ctypes mirrors in slamhot/__init__.py agree with include/slamhot.h: every field's offset
and every struct's size, as gcc lays the C header out (host logic; no GPU)."""
import ctypes as C
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-slam3-noted_amd"))

PAIRS = {"OrbParams": "slam_orb_params", "BowSide": "slam_bow_side", "FrameView": "slam_frame_view",
         "LastFrameView": "slam_last_frame", "KFPointsView": "slam_kf_points", "Camera": "slam_camera",
         "LbaProblem": "slam_lba_problem", "LbaOptions": "slam_lba_options", "LbaResult": "slam_lba_result",
         "PoseFrame": "slam_pose_frame", "PoseResult": "slam_pose_result", "TriKF": "slam_tri_kf",
         "TriPair": "slam_tri_pair", "TrackerConfig": "slam_tracker_config", "TrackRecord": "slam_track_record",
         "TrackKeyFrame": "slam_track_keyframe", "TrackState": "slam_track_state",
         "TrackFrame": "slam_track_frame"}


@pytest.fixture(scope="module")
def c_layout(tmp_path_factory):
    import slamhot
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "slamhot.h"', "int main(void) {"]
    for py, cn in PAIRS.items():
        cls = getattr(slamhot, py)
        lines.append(f'  printf("{py} size %zu\\n", sizeof({cn}));')
        for f in cls._fields_:
            lines.append(f'  printf("{py} {f[0]} %zu\\n", offsetof({cn}, {f[0]}));')
    lines += ["  return 0;", "}"]
    d = tmp_path_factory.mktemp("abi")
    src, exe = d / "layout.c", d / "layout"
    src.write_text("\n".join(lines) + "\n")
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    return {tuple(l.split()[:2]): int(l.split()[2]) for l in out.splitlines()}


@pytest.mark.parametrize("py", sorted(PAIRS))
def test_struct_layout_matches_header(c_layout, py):
    import slamhot
    cls = getattr(slamhot, py)
    assert C.sizeof(cls) == c_layout[(py, "size")], f"{py}: sizeof differs from {PAIRS[py]}"
    for f in cls._fields_:
        assert getattr(cls, f[0]).offset == c_layout[(py, f[0])], f"{py}.{f[0]} offset"
