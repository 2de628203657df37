"""Per-kernel register / spill / scratch / occupancy table of one HIP translation unit (hipcc's
-Rpass-analysis=kernel-resource-usage remarks), demangled.  Diagnostic only.

    python tools/resource_usage.py insite_refine.hip [-DFLAG=V ...] [--grep PATTERN]
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ode-discovery-for-longitudinal-heterogeneous-treatment-effects-inference_amd")


def main():
    args = sys.argv[1:]
    pat = None
    if "--grep" in args:
        i = args.index("--grep")
        pat = args[i + 1]
        del args[i:i + 2]
    tu, flags = args[0], args[1:]
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", *flags, "-I",
           os.path.join(ROOT, "include"), "-c", "-o", "/tmp/_ru.o", os.path.join(PKG, "csrc", tu),
           "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark:\s+(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|"
                      r"SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]|SGPRs): (\S+)", line)
        if not m:
            continue
        k, v = m.group(1), m.group(2)
        if k == "Function Name":
            cur = {"name": v}
            rows.append(cur)
        elif cur is not None:
            cur[k.split(" [")[0]] = v
    names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows),
                           capture_output=True, text=True).stdout.splitlines()
    print(f"{'VGPR':>5} {'AGPR':>5} {'SGPR':>5} {'vspill':>6} {'sspill':>6} {'scratch':>7} {'occ':>3} {'LDS':>6}  kernel")
    for r, n in zip(rows, names):
        n = re.sub(r"\(anonymous namespace\)::", "", n)
        n = re.sub(r"\(.*\)$", "", n)
        if pat and not re.search(pat, n):
            continue
        print(f"{r.get('VGPRs', '?'):>5} {r.get('AGPRs', '?'):>5} {r.get('SGPRs', '?'):>5} {r.get('VGPRs Spill', '?'):>6} "
              f"{r.get('SGPRs Spill', '?'):>6} {r.get('ScratchSize', '?'):>7} {r.get('Occupancy', '?'):>3} "
              f"{r.get('LDS Size', '?'):>6}  {n}")


if __name__ == "__main__":
    main()
