"""Exactly rounded float32 helpers for the independent numpy restatements in tests/ (numpy has no
fused multiply-add): fmaf(a, b, c) = a*b+c rounded once, via rational arithmetic."""
from fractions import Fraction

import numpy as np


def f32_round(q: Fraction) -> np.float32:
    """A rational rounded once to float32 (round half to even; normal range)."""
    if q == 0:
        return np.float32(0.0)
    neg, q = q < 0, abs(q)
    e = q.numerator.bit_length() - q.denominator.bit_length()
    if Fraction(2) ** e > q:
        e -= 1
    m = round(q * Fraction(2) ** (23 - e))  # round() on a Fraction is half-to-even
    v = np.float32(float(Fraction(m) * Fraction(2) ** (e - 23)))
    return -v if neg else v


def fmaf(a, b, c) -> np.float32:
    return f32_round(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c)))


def chain3(a, b):
    """cv::Matx row . column as compiled: fma chain from +0."""
    return fmaf(a[2], b[2], fmaf(a[1], b[1], fmaf(a[0], b[0], np.float32(0))))


def norm_d(v):
    """cv::norm(Matx31f): squares of the floats summed in double, sqrt, rounded to float."""
    x, y, z = (float(t) for t in v)
    return np.float32(np.sqrt((x * x + y * y) + z * z))
