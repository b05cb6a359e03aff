"""Register / spill / occupancy table of the kernels in one HIP source (CPU).

    python tools/kernel_regs.py fd_kernels.hip [name-regex]

Compiles the source for gfx950 with the library's flags and
-Rpass-analysis=kernel-resource-usage (the same figures the code object's
notes carry) and prints one line per kernel.
"""
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dynamic-video-compression-surveillance_amd", "csrc")


def main():
    src = os.path.join(CSRC, sys.argv[1])
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    extra = sys.argv[3:]
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC",
                        "-ffp-contract=off", "-c", "--offload-device-only", "-Rpass-analysis=kernel-resource-usage",
                        *extra, src, "-o", "/tmp/_kregs.o"], capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr[-4000:])
    rows, cur = {}, None
    for line in r.stderr.split("\n"):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            rows[cur] = {}
            continue
        m = re.search(r"remark:\s+(TotalSGPRs|VGPRs|AGPRs|SGPRs Spill|VGPRs Spill|Occupancy \[waves/SIMD\]|"
                      r"LDS Size \[bytes/block\]|ScratchSize \[bytes/lane\]): (\d+)", line)
        if m and cur:
            rows[cur][m.group(1)] = int(m.group(2))
    names = list(rows)
    filt = shutil.which("c++filt")
    dem = subprocess.run([filt], input="\n".join(names), capture_output=True, text=True).stdout.split("\n") \
        if filt else names
    for n, d in zip(names, dem):
        d = re.sub(r"\(.*", "", d)
        if pat and not pat.search(d):
            continue
        x = rows[n]
        print(f"{d:64s} vgpr {x.get('VGPRs')} sgpr {x.get('TotalSGPRs')} sgpr_spill {x.get('SGPRs Spill')} "
              f"vgpr_spill {x.get('VGPRs Spill')} scratch {x.get('ScratchSize [bytes/lane]')} "
              f"lds {x.get('LDS Size [bytes/block]')} occ {x.get('Occupancy [waves/SIMD]')}")


if __name__ == "__main__":
    main()
