"""ISA audit of the exact kernels: compile csrc/dlsim_abi.hip
for gfx950 with --save-temps and count, per element policy, the fused
multiply-add (v_fma*/v_fmac*/v_mad_f32) and mixed-precision (v_*_mix*)
instructions. Exact policies must have none: the reference rounds every
product and every sum separately. (The mean policies' FMAs are the IEEE
division sequence; FAST policies fuse by design.)

    python scripts/audit_isa.py > profiles/r01_isa_audit.json
"""
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "decentralized-learning-simulator_amd", "csrc")
POLICIES = ("BF16Exact", "BF16Fast", "BF16Mean", "F16Exact", "F16Fast", "F16Mean", "F32Exact", "F32Fast",
            "F32Mean")


def main():
    with tempfile.TemporaryDirectory() as d:
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "-fPIC", "-I", os.path.join(ROOT, "include"), "-I", CSRC, "-c",
                        os.path.join(CSRC, "dlsim_abi.hip"), "-o", os.path.join(d, "abi.o"), "--save-temps"],
                       cwd=d, check=True, stderr=subprocess.DEVNULL)
        s = open(os.path.join(d, "dlsim_abi-hip-amdgcn-amd-amdhsa-gfx950.s")).read()
    stats = {}
    for m in re.finditer(r"^(_Z\S+):", s, re.M):
        name = m.group(1)
        body = s[m.end():s.find("s_endpgm", m.end())]
        # Itanium mangling prefixes every name with its length: 9BF16Exact, 8F16Exact
        key = next((k for k in POLICIES if f"{len(k)}{k}" in name), None)
        if key is None:
            continue
        e = stats.setdefault(key, {"kernels": 0, "fma": 0, "mix": 0})
        e["kernels"] += 1
        e["fma"] += len(re.findall(r"\bv_(pk_)?fmac?_f32\b|\bv_mad_f32\b", body))
        e["mix"] += len(re.findall(r"_mix", body))
    bad = {k: v for k, v in stats.items() if k.endswith("Exact") and (v["fma"] or v["mix"])}
    print(json.dumps({"target": "gfx950", "per_policy": stats, "exact_policies_clean": not bad}, indent=1))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
