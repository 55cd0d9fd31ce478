"""EuRoC I/O around the hot path: the stereo example's image list loader
(stereo_euroc.cc:246-270), the OpenCV-YAML settings it reads (stereo_euroc.cc:84-112), the
rectification maps (cv::initUndistortRectifyMap, stereo_euroc.cc:117-118) with the device
remap (slamhot_rectify_batch_device, stereo_euroc.cc:168-169), and the trajectory writer
System::SaveTrajectoryEuRoC (System.cc:514-611).

initUndistortRectifyMap is restated from OpenCV 4.2.0's published algorithm
(undistort.dispatch.cpp: incremental row walk in double, rational + tangential + thin-prism
model, identity tilt); OpenCV is not in this image, so its bit-parity is unpinned.  The device
remap is bit-exact against oracle/rectify_oracle.cpp on any float maps.
"""
from __future__ import annotations

import ctypes as C
import re
from pathlib import Path

import numpy as np


# --------------------------------------------------------------------------- image lists
def LoadImages(path_left: str, path_right: str, path_times: str):
    """stereo_euroc.cc LoadImages: one line per frame holding the nanosecond timestamp;
    images are <path>/<line>.png, timestamps line / 1e9 (seconds)."""
    left, right, times = [], [], []
    for line in Path(path_times).read_text().splitlines():
        if not line:
            continue
        left.append(f"{path_left}/{line}.png")
        right.append(f"{path_right}/{line}.png")
        tok = line.split()
        times.append(float(tok[0]) / 1e9 if tok else 0.0)
    return left, right, times


# --------------------------------------------------------------------------- settings
_MAT = re.compile(r"^(?P<key>[\w.]+):\s*!!opencv-matrix\s*$")


def read_settings(path: str) -> dict:
    """The subset of cv::FileStorage YAML the EuRoC settings use: `key: scalar` lines and
    `key: !!opencv-matrix` blocks (rows, cols, dt, data: [...], data may span lines)."""
    out: dict = {}
    lines = Path(path).read_text().splitlines()
    i = 0
    while i < len(lines):
        raw = lines[i].split("#", 1)[0].rstrip()
        i += 1
        if not raw.strip() or raw.startswith("%YAML") or raw.strip() == "---":
            continue
        m = _MAT.match(raw.strip())
        if m:
            block = {}
            body = ""
            while i < len(lines) and (lines[i].startswith((" ", "\t")) or not lines[i].strip()):
                body += " " + lines[i].split("#", 1)[0]
                i += 1
            for k in ("rows", "cols"):
                block[k] = int(re.search(rf"\b{k}:\s*(\d+)", body).group(1))
            data = re.search(r"data:\s*\[([^\]]*)\]", body, re.S).group(1)
            vals = [float(v) for v in data.replace("\n", " ").split(",") if v.strip()]
            out[m.group("key")] = np.array(vals, np.float64).reshape(block["rows"], block["cols"])
            continue
        if ":" in raw:
            k, v = raw.split(":", 1)
            v = v.strip().strip('"')
            try:
                out[k.strip()] = int(v) if re.fullmatch(r"[-+]?\d+", v) else float(v)
            except ValueError:
                out[k.strip()] = v
    return out


# --------------------------------------------------------------------------- rectification
def init_undistort_rectify_map(K, D, R, P, size):
    """cv::initUndistortRectifyMap(K, D, R, P(0:3, 0:3), Size(w, h), CV_32F) -> (map_x, map_y)."""
    w, h = size
    A = np.asarray(K, np.float64).reshape(3, 3)
    Ar = np.asarray(P, np.float64).reshape(3, -1)[:, :3]
    Rm = np.asarray(R, np.float64).reshape(3, 3)
    d = np.zeros(14)
    dv = np.asarray(D, np.float64).ravel()
    d[: len(dv)] = dv
    k1, k2, p1, p2 = d[:4]
    k3 = d[4] if len(dv) >= 5 else 0.0
    k4, k5, k6 = (d[5], d[6], d[7]) if len(dv) >= 8 else (0.0, 0.0, 0.0)
    s1, s2, s3, s4 = d[8:12] if len(dv) >= 12 else (0.0, 0.0, 0.0, 0.0)
    ir = np.linalg.inv(Ar @ Rm).ravel()
    u0, v0, fx, fy = A[0, 2], A[1, 2], A[0, 0], A[1, 1]
    mx = np.empty((h, w), np.float32)
    my = np.empty((h, w), np.float32)
    # the row walk accumulates _x += ir[0] per column: a cumulative sum, evaluated sequentially
    cols = np.arange(w)
    for i in range(h):
        _x = np.empty(w)
        _y = np.empty(w)
        _w = np.empty(w)
        x0, y0, w0 = i * ir[1] + ir[2], i * ir[4] + ir[5], i * ir[7] + ir[8]
        for arr, start, step in ((_x, x0, ir[0]), (_y, y0, ir[3]), (_w, w0, ir[6])):
            acc = start
            for j in cols:
                arr[j] = acc
                acc += step
        ww = 1.0 / _w
        x = _x * ww
        y = _y * ww
        x2, y2 = x * x, y * y
        r2 = x2 + y2
        _2xy = 2 * x * y
        kr = (1 + ((k3 * r2 + k2) * r2 + k1) * r2) / (1 + ((k6 * r2 + k5) * r2 + k4) * r2)
        xd = x * kr + p1 * _2xy + p2 * (r2 + 2 * x2) + s1 * r2 + s2 * r2 * r2
        yd = y * kr + p1 * (r2 + 2 * y2) + p2 * _2xy + s3 * r2 + s4 * r2 * r2
        mx[i] = (fx * 1.0 * xd + u0).astype(np.float32)
        my[i] = (fy * 1.0 * yd + v0).astype(np.float32)
    return mx, my


class Rectifier:
    """Device cv::remap(INTER_LINEAR) for one camera's maps (slamhot_rectifier_*)."""

    def __init__(self, map_x, map_y, src_size=None, device: int = 0):
        from . import I, P, check, lib
        L = lib()
        if not getattr(L, "_rect_ready", False):
            L.slamhot_rectifier_create.argtypes = [I, I, I, I, I, P, P, C.POINTER(P)]
            L.slamhot_rectifier_destroy.argtypes = [P]
            L.slamhot_rectifier_destroy.restype = None
            L.slamhot_rectify_batch_device.argtypes = [P, I, P, I, C.c_int64, P, I, C.c_int64, P]
            L._rect_ready = True
        self.map_x = np.ascontiguousarray(map_x, np.float32)
        self.map_y = np.ascontiguousarray(map_y, np.float32)
        self.dh, self.dw = self.map_x.shape
        self.sw, self.sh = src_size or (self.dw, self.dh)
        h = P()
        check(L.slamhot_rectifier_create(device, self.sw, self.sh, self.dw, self.dh, self.map_x.ctypes.data,
                                         self.map_y.ctypes.data, C.byref(h)), "rectifier_create")
        self._h = h

    def close(self):
        from . import lib
        if getattr(self, "_h", None):
            lib().slamhot_rectifier_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def rectify_batch_device(self, nframes, d_src, src_pitch, src_stride, d_dst, dst_pitch, dst_stride, stream=None):
        from . import P, check, lib
        check(lib().slamhot_rectify_batch_device(self._h, nframes, P(d_src), src_pitch, src_stride, P(d_dst), dst_pitch,
                                                 dst_stride, P(stream) if stream else None), "rectify_batch_device")

    def __call__(self, images):
        """Host convenience: (n, sh, sw) or (sh, sw) u8 -> rectified u8 (torch for device buffers)."""
        import torch
        im = np.ascontiguousarray(images, np.uint8)
        single = im.ndim == 2
        if single:
            im = im[None]
        dev = torch.device("cuda", torch.cuda.current_device())
        d_src = torch.from_numpy(im).to(dev)
        d_dst = torch.empty((len(im), self.dh, self.dw), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        self.rectify_batch_device(len(im), d_src.data_ptr(), self.sw, self.sw * self.sh, d_dst.data_ptr(), self.dw,
                                  self.dw * self.dh)
        torch.cuda.synchronize()
        out = d_dst.cpu().numpy()
        return out[0] if single else out


# --------------------------------------------------------------------------- trajectory
def _quat_from_R(M):
    """Eigen::Quaterniond(const Matrix3d&) (Quaternion.h: quaternionbase_assign_impl) -> x, y, z, w."""
    t = M[0, 0] + M[1, 1] + M[2, 2]
    q = np.zeros(4)
    if t > 0:
        t = np.sqrt(t + 1.0)
        q[3] = 0.5 * t
        t = 0.5 / t
        q[0] = (M[2, 1] - M[1, 2]) * t
        q[1] = (M[0, 2] - M[2, 0]) * t
        q[2] = (M[1, 0] - M[0, 1]) * t
    else:
        i = 0
        if M[1, 1] > M[0, 0]:
            i = 1
        if M[2, 2] > M[i, i]:
            i = 2
        j = (i + 1) % 3
        k = (j + 1) % 3
        t = np.sqrt(M[i, i] - M[j, j] - M[k, k] + 1.0)
        q[i] = 0.5 * t
        t = 0.5 / t
        q[3] = (M[k, j] - M[j, k]) * t
        q[j] = (M[j, i] + M[i, j]) * t
        q[k] = (M[k, i] + M[i, k]) * t
    return q


def save_trajectory_euroc(filename: str, timestamps, Tcw_list):
    """System::SaveTrajectoryEuRoC, visual case (System.cc:597-603): per frame
    `1e9*t` (fixed, 6 decimals) then twc and the quaternion of Rwc (x y z w), fixed 9 decimals.
    Tcw_list holds the final camera poses (Tcw = (*lit) * Trw), float 4x4."""
    with open(filename, "w") as f:
        for t, T in zip(timestamps, Tcw_list):
            T = np.asarray(T, np.float32).reshape(4, 4)
            Rwc = T[:3, :3].T.copy()
            # twc = -Rwc * tcw as a cv::Mat product (double accumulation, rounded once)
            twc = (-(Rwc.astype(np.float64) @ T[:3, 3].astype(np.float64))).astype(np.float32)
            q = _quat_from_R(Rwc.astype(np.float64)).astype(np.float32)
            f.write(f"{1e9 * t:.6f} {twc[0]:.9f} {twc[1]:.9f} {twc[2]:.9f} {q[0]:.9f} {q[1]:.9f} {q[2]:.9f} "
                    f"{q[3]:.9f}\n")
