"""Per-kernel registers, scratch, occupancy and LDS of ngs_kernels.hip for gfx950 (diagnostic).

Compiles the device side with -Rpass-analysis=kernel-resource-usage and prints one line per
ngs kernel. usage: python tools/kernel_resources.py [source.hip] [extra hipcc flags...]
"""
import re
import subprocess
import sys
import tempfile

SRC = sys.argv[1] if len(sys.argv) > 1 else "stringsearchlib_amd/csrc/ngs_kernels.hip"
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fhip-fp32-correctly-rounded-divide-sqrt",
         "--cuda-device-only", "-c", "-Rpass-analysis=kernel-resource-usage"] + sys.argv[2:]
with tempfile.TemporaryDirectory() as d:
    res = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, SRC, "-o", f"{d}/k.co"], capture_output=True, text=True)
rows, cur = {}, None
for line in res.stderr.splitlines():
    m = re.search(r"remark: (?:\s*)([^:]+): (\S+) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2)
    if k == "Function Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
names = subprocess.run(["c++filt"], input="\n".join(rows), capture_output=True, text=True).stdout.splitlines()
for (mangled, r), dn in zip(rows.items(), names):
    if "ngs" not in mangled:
        continue
    dn = dn.replace("ngs::(anonymous namespace)::", "").replace("ngs::", "")
    dn = re.sub(r"\(.*", "", dn.replace("void ", "", 1))
    print(f"{dn[:64]:64s} VGPR {r.get('VGPRs', '?'):>4} AGPR {r.get('AGPRs', '?'):>3} scratch {r.get('ScratchSize [bytes/lane]', '?'):>4} "
          f"occ {r.get('Occupancy [waves/SIMD]', '?'):>2} vspill {r.get('VGPRs Spill', '?'):>3} sspill {r.get('SGPRs Spill', '?'):>3} "
          f"lds {r.get('LDS Size [bytes/block]', '?')}")
if res.returncode:
    print(res.stderr[-2000:], file=sys.stderr)
    sys.exit(res.returncode)
