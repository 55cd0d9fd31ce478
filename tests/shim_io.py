"""Binary exchange with tests/cpp/shim_driver (the drop-in shim bodies of
include/slamhot_orbslam3.hpp on ORB-SLAM3 stand-ins).  The map written here is the one the
Python mirror (slamhot.optimizer) holds, so both sides start from identical objects."""
from __future__ import annotations

import os
import struct
import subprocess
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
DRIVER = Path(os.environ.get("SLAMHOT_SHIM_DRIVER", str(ROOT / "tests" / "cpp" / "shim_driver")))  # sanitizer builds: tools/sanitize.sh


def write_map(path, pmap, kfs, mps, cur_index=-1):
    """kfs: the mirror's KeyFrames with mnId == index; mps: MapPoints with mnId == index."""
    from slamhot.synth import _level_tables
    _, isig, _ = _level_tables()
    k0 = kfs[0]
    rig = k0.mpCamera2 is not None
    obs = []
    for pi, mp in enumerate(mps):
        for k, (li, ri) in mp.GetObservations().items():
            obs.append((k.mnId, pi, li, ri))
    b = bytearray()
    cur = cur_index % len(kfs)
    b += struct.pack("<7i", len(kfs), len(mps), len(obs), pmap.GetInitKFid(), cur, int(pmap.IsInertial()), int(rig))
    b += struct.pack("<5f", k0.fx, k0.fy, k0.cx, k0.cy, k0.mbf)
    b += struct.pack("<4f", *(k0.mpCamera2 if rig else (0, 0, 0, 0)))
    b += np.asarray(k0.mTrl if rig else np.eye(4), np.float32).tobytes()
    b += np.asarray(isig, np.float32).tobytes()
    for k in kfs:
        nr = len(k.mvKeysRight) if rig else 0
        b += struct.pack("<3i", k.mnId, len(k.mvKeysUn), nr)
        b += np.asarray(k.Tcw, np.float32).tobytes()
        for i in range(len(k.mvKeysUn)):
            kp = k.mvKeysUn[i]
            b += struct.pack("<ffif", kp["x"], kp["y"], int(kp["octave"]), k.mvuRight[i])
        for i in range(nr):
            kp = k.mvKeysRight[i]
            b += struct.pack("<ffi", kp["x"], kp["y"], int(kp["octave"]))
    for mp in mps:
        b += struct.pack("<i", mp.mnId) + np.asarray(mp.pos, np.float32).tobytes()
    for o in obs:
        b += struct.pack("<4i", *o)
    cov = kfs[cur].covisible
    b += struct.pack("<i", len(cov)) + np.asarray([k.mnId for k in cov], np.int32).tobytes()
    Path(path).write_bytes(bytes(b))


class Blob:
    def __init__(self, data: bytes):
        self.d, self.p = data, 0

    def i32(self):
        v = struct.unpack_from("<i", self.d, self.p)[0]
        self.p += 4
        return v

    def vec(self, dt):
        n = self.i32()
        dt = np.dtype(dt)
        a = np.frombuffer(self.d, dt, n, self.p).copy()
        self.p += n * dt.itemsize
        return a


def run(mode, inp, out):
    r = subprocess.run([str(DRIVER), mode, str(inp), str(out)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    return Blob(Path(out).read_bytes())


def read_flatten(b: Blob):
    ok, nf, nloc, nmp = b.i32(), b.i32(), b.i32(), b.i32()
    out = dict(ok=ok, num_fixed=nf, num_local=nloc, num_mps=nmp, kf_ids=b.vec("<i4"), mp_ids=b.vec("<i4"))
    for k, dt in (("kf_Tcw", "<f4"), ("kf_fixed", "u1"), ("pt_pos", "<f4"), ("edge_pt", "<i4"), ("edge_kf", "<i4"),
                  ("edge_obs", "<f4"), ("edge_inv_sigma2", "<f4"), ("edge_body", "u1"), ("kf_Trl", "<f4")):
        out[k] = b.vec(dt)
    return out


class Out:
    """Little-endian writer for the shim_driver input files."""

    def __init__(self):
        self.b = bytearray()

    def i32(self, *v):
        self.b += struct.pack(f"<{len(v)}i", *[int(x) for x in v])
        return self

    def f32(self, *v):
        self.b += struct.pack(f"<{len(v)}f", *[float(x) for x in v])
        return self

    def raw(self, a, dt=None):
        a = np.ascontiguousarray(a if dt is None else np.asarray(a, dt))
        self.b += a.tobytes()
        return self

    def save(self, path):
        Path(path).write_bytes(bytes(self.b))
        return path


def level_tables(nlevels=8, scale_factor=1.2):
    """mvScaleFactors / mvInvLevelSigma2 / mfLogScaleFactor as ORBextractor / Frame compute them
    (ORBextractor.cc:413-425, Frame.cc:107-113): the oracle's own tables."""
    import oracle_bind as ob
    sc, isc, s2, is2, _ = ob.levels(ob.params(nlevels=nlevels, scale=scale_factor))
    lsf = np.float32(np.log(np.float64(np.float32(scale_factor))))
    return sc, is2, lsf


def write_frame(o: Out, fv, kps_un, kps, uright, desc, state, bad, Tcw, mnId=7):
    """A stand-in Frame for shim_driver (read_frame): fv is the slam_frame_view the oracle is given
    for the same Frame (its bounds, grid, camera and scale tables are written from it)."""
    import ctypes as C
    n = len(kps_un)
    o.i32(n, mnId).raw(Tcw, np.float32)
    o.f32(fv.fx, fv.fy, fv.cx, fv.cy, fv.bf, fv.b)
    o.f32(fv.min_x, fv.min_y, fv.max_x, fv.max_y, fv.grid_inv_w, fv.grid_inv_h)
    sc = np.ctypeslib.as_array(C.cast(fv.scale, C.POINTER(C.c_float)), (fv.nlevels,)).copy()
    _, is2, _ = level_tables(fv.nlevels)
    o.i32(fv.nlevels).raw(sc, np.float32).f32(fv.log_scale).raw(is2, np.float32)
    rec = np.zeros(n, np.dtype([("ku", "V28"), ("k", "V28"), ("ur", "<f4"), ("d", "u1", 32), ("st", "i1"), ("bad", "u1")]))
    rec["ku"] = np.ascontiguousarray(kps_un).view("V28")
    rec["k"] = np.ascontiguousarray(kps).view("V28")
    rec["ur"] = uright
    rec["d"] = desc
    rec["st"] = state
    rec["bad"] = bad
    o.raw(rec)
    return o


def run_any(mode, out: Out, tmp_path, name="in.bin"):
    return run(mode, out.save(Path(tmp_path) / name), Path(tmp_path) / (name + ".out"))
