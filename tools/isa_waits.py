"""Serialized-load finder: compiles a HIP source to gfx950 assembly and lists, per kernel, global / buffer loads
whose result is waited for (s_waitcnt vmcnt(0)) within the next few instructions -- each such load costs a full
memory round trip of the kernel's dependency chain.  Usage: python tools/isa_waits.py graph-transformer_amd/csrc/X.hip"""
import os
import re
import subprocess
import sys
import tempfile

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(src, window=4, min_count=2):
    out = os.path.join(tempfile.mkdtemp(), "k.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-slp-vectorize",
                    f"-I{R}/include", f"-I{R}/graph-transformer_amd/csrc", "--offload-device-only", "-S", "-o", out, src],
                   check=True, capture_output=True)
    s = open(out).read()
    for m in re.finditer(r"^(_ZN\S+):", s, re.M):
        end = s.find(".Lfunc_end", m.end())
        lines = [ln.strip() for ln in s[m.end():end].splitlines()]
        bad = 0
        for k, ln in enumerate(lines):
            if ln.startswith(("global_load", "buffer_load")):
                if any(q.startswith("s_waitcnt vmcnt(0)") for q in lines[k + 1:k + 1 + window]):
                    bad += 1
        if bad >= min_count:
            name = subprocess.run(["c++filt", m.group(1)], capture_output=True, text=True).stdout.strip()
            print(f"{bad:4d}  {name[:120]}")


if __name__ == "__main__":
    main(sys.argv[1])
