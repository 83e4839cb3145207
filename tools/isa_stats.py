#!/usr/bin/env python3
"""Per-kernel resource usage and instruction mix of a standalone gfx950 compile.

Compile one source with the resource remarks and the assembly kept, e.g.

  hipcc --offload-arch=gfx950 -O3 -std=c++17 -c fm_bwd.hip --save-temps \\
        -Rpass-analysis=kernel-resource-usage 2> res.txt

then: python tools/isa_stats.py res.txt fm_bwd-hip-amdgcn-amd-amdhsa-gfx950.s [name-substring ...]

Prints VGPRs / SGPRs / occupancy / spills and the static instruction counts (all, global loads,
ds_bpermute, 64-bit address arithmetic, SGPR-spill lane moves) of every kernel whose mangled name
contains one of the substrings.
"""
import re
import subprocess
import sys


def resources(path):
    cur, out = None, {}
    for line in open(path):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"remark: \S+\s+(.+?): (\S+) \[-Rpass", line)
        if m and cur:
            out[cur][m.group(1).strip()] = m.group(2)
    return out


def body(asm, f):
    i = asm.find("\n" + f + ":")
    j = asm.find(".Lfunc_end", i)
    return [ln.strip() for ln in asm[i:j].splitlines()[1:] if ln.startswith("\t") and not ln.startswith("\t.")
            and not ln.startswith("\t;")]


def main():
    res = resources(sys.argv[1])
    asm = open(sys.argv[2]).read()
    pats = sys.argv[3:] or [""]
    print(f"{'kernel':64s} {'VGPR':>4} {'SGPR':>4} {'occ':>3} {'sspill':>6} {'vspill':>6} {'inst':>5} {'gload':>5} "
          f"{'bperm':>5} {'mad64':>5} {'lane':>4}")
    for f, d in res.items():
        if not any(p in f for p in pats):
            continue
        b = body(asm, f)
        dm = subprocess.run(["c++filt", f], capture_output=True, text=True).stdout.strip()
        dm = re.sub(r"^void |\(.*$", "", dm)
        cnt = lambda rx: sum(1 for ln in b if re.match(rx, ln))  # noqa: E731
        print(f"{dm[:64]:64s} {d.get('VGPRs', '?'):>4} {d.get('TotalSGPRs', '?'):>4} "
              f"{d.get('Occupancy [waves/SIMD]', '?'):>3} {d.get('SGPRs Spill', '?'):>6} "
              f"{d.get('VGPRs Spill', '?'):>6} "
              f"{len(b):>5} {cnt(r'global_load'):>5} {cnt(r'ds_bpermute'):>5} "
              f"{cnt(r'v_(mad_u64_u32|mad_i64_i32|lshl_add_u64|add_co_u32)'):>5} {cnt(r'v_(readlane|writelane)'):>4}")


if __name__ == "__main__":
    main()
