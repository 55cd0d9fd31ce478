"""Extract the 256-pair rBRIEF sampling pattern as a DATA file.

Provenance: the table is the learned ORB test pattern (Rublee et al. 2011, OpenCV
features2d/src/orb.cpp, BSD) that ORB-SLAM3 embeds as `bit_pattern_31_`
(/root/reference/src/ORBextractor.cc:148-406).  Bit-exact descriptors need the exact
integers, so this script reads the 1024 integers out of the reference file once and
writes them as a bare comma-separated list (no code) to
orb-slam3-noted_amd/csrc/orb_pattern.inc.  The generated file is committed because the
GPU box has no /root/reference.
"""
import re
import sys
from pathlib import Path

SRC = Path("/root/reference/src/ORBextractor.cc")
OUT = Path(__file__).resolve().parents[1] / "orb-slam3-noted_amd" / "csrc" / "orb_pattern.inc"


def main():
    text = SRC.read_text()
    start = text.index("bit_pattern_31_[256*4]")
    body = text[text.index("{", start) + 1: text.index("};", start)]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    vals = [int(v) for v in re.findall(r"-?\d+", body)]
    assert len(vals) == 1024, len(vals)
    lines = ["/* ORB rBRIEF pattern: 256 pairs (x0,y0,x1,y1), data only; see tools/extract_pattern.py */"]
    for i in range(256):
        lines.append("%d,%d,%d,%d," % tuple(vals[4 * i: 4 * i + 4]))
    OUT.write_text("\n".join(lines) + "\n")
    print("wrote", OUT, file=sys.stderr)


if __name__ == "__main__":
    main()
