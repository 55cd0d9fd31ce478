#!/usr/bin/env python3
"""Study tool (runs in the build container only, never on the GPU box): list the scalar
floating-point instructions of one function of a reference object file, read as DATA with
`objdump -d` (nothing from the reference is executed or linked).

    python3 tools/disasm/fp_sites.py <object.o> '<demangled-name substring>' [--all]

It prints every FMA / float / double arithmetic instruction with its offset, so that each
contraction GCC 9.3 made under -O3 -march=native (reference evaluation/CMakeFiles/.../flags.make:5)
can be restated with an explicit fmaf/fma in oracle/ and csrc/.  DESIGN.md §1 lists the sites.
"""
import re
import subprocess
import sys

FP = re.compile(r"\bv(fn?m(add|sub)\d{3}s[sd]|(add|sub|mul|div|sqrt|min|max)s[sd]|cvt\w+|rndscale\w+|u?comis[sd]|xorp[sd]|andp[sd])\b")


def functions(obj):
    out = subprocess.run(["objdump", "-d", "-C", "-r", "--no-show-raw-insn", "-j", ".text", obj],
                         capture_output=True, text=True, check=True).stdout
    cur, body = None, []
    for line in out.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.*)>:$", line)
        if m:
            if cur:
                yield cur, body
            cur, body = (int(m.group(1), 16), m.group(2)), []
        elif cur:
            body.append(line)
    if cur:
        yield cur, body


def main():
    obj, pat = sys.argv[1], sys.argv[2]
    show_all = "--all" in sys.argv
    for (addr, name), body in functions(obj):
        if pat not in name:
            continue
        n_fma = sum(1 for l in body if re.search(r"\bvfn?m(add|sub)\d{3}s[sd]\b", l))
        print(f"== {name} @0x{addr:x}: {n_fma} scalar FMA")
        for l in body:
            if show_all or FP.search(l) or "call" in l or "R_X86_64_PLT32" in l:
                print(l)


if __name__ == "__main__":
    main()
