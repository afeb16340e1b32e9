"""Compact per-kernel register / occupancy report from hipcc's
-Rpass-analysis=kernel-resource-usage remarks.

usage: python tools/kernel_resources.py paig_reproduction_amd/csrc/conv_mfma.hip [filter] [-DNAME=VALUE ...]
"""
import re
import subprocess
import sys


def main():
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    defs = [a for a in sys.argv[3:] if a.startswith("-D")]   # A/B build macros
    out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-c", src, "-o",
                          "/dev/null", "-Rpass-analysis=kernel-resource-usage"] + defs, capture_output=True, text=True).stderr
    cur = None
    rows = {}
    for line in out.splitlines():
        m = re.search(r"remark: (.*?) \[-Rpass", line)
        if not m:
            continue
        msg = m.group(1)
        if msg.startswith("Function Name:"):
            cur = msg.split(":", 1)[1].strip()
            try:
                cur = subprocess.run(["c++filt", cur], capture_output=True, text=True).stdout.strip()
            except OSError:
                pass
            cur = re.sub(r"\(.*", "", re.sub(r"\(anonymous namespace\)::", "", cur)).replace("void ", "")
            rows[cur] = {}
        elif cur is not None and ":" in msg:
            k, v = msg.split(":", 1)
            rows[cur][k.strip()] = v.strip()
    for k, r in rows.items():
        if filt in k:
            print("%-62s vgpr=%-4s agpr=%-3s spill=%s/%s occ=%s lds=%s" % (
                k[:62], r.get("VGPRs"), r.get("AGPRs"), r.get("VGPRs Spill"), r.get("SGPRs Spill"),
                r.get("Occupancy [waves/SIMD]"), r.get("LDS Size [bytes/block]")))


if __name__ == "__main__":
    main()
