"""ISA audit of the exact kernels, on the BUILT library.

Extracts the gfx950 code objects from the `.hip_fatbin` section of
`libdlsim_hip.so` (every translation unit: the C ABI and the inst_*.hip
instantiation units), disassembles them with llvm-objdump and counts, per
kernel, the fused multiply-add (v_fma*/v_fmac*/v_mad_f32/v_pk_fma*) and
mixed-precision (v_*_mix*) instructions. The exact element policies must have
none: the reference rounds every product and every sum separately
(fedavg.py:25). The mean policies' FMAs are the IEEE division
sequence; FAST policies fuse by design; the chunk-mean kernels are plain adds.

    python scripts/audit_isa.py [lib.so] > profiles/r03_isa_audit.json

tests/test_isa_audit.py runs the same audit in the CPU suite.
"""
import json
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "decentralized-learning-simulator_amd", "dasklearn_amd", "lib", "libdlsim_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"
POLICIES = ("BF16Exact", "BF16Fast", "BF16Mean", "F16Exact", "F16Fast", "F16Mean", "F32Exact", "F32Fast",
            "F32Mean", "F64Exact", "F64Fast", "MixedSlots")
# exact like the *Exact policies: the mixed-dtype fold (k_wreduce_mixed, round 5)
EXACT_KEYS = tuple(k for k in POLICIES if k.endswith("Exact")) + ("MixedSlots",)
# encodings are suffixed in the disassembly (v_fmac_f32_e32, v_fma_f32_e64)
FMA_RE = re.compile(r"\bv_(pk_)?(fmac?|mac|mad|fma_legacy|fmac_legacy)_f(32|64)(_e(32|64|64_dpp|32_dpp))?\b")
MIX_RE = re.compile(r"\bv_\w*_mix\w*\b")
# register spills (gfx950 spills through scratch_* instructions)
SPILL_RE = re.compile(r"\bscratch_(load|store)_\w+")
BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _section(path, name):
    """Bytes of ELF section `name` (64-bit little-endian ELF)."""
    with open(path, "rb") as f:
        data = f.read()
    if data[:4] != b"\x7fELF" or data[4] != 2:
        raise ValueError(f"{path}: not a 64-bit ELF")
    shoff, = struct.unpack_from("<Q", data, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", data, 0x3A)
    def sh(i):
        return struct.unpack_from("<IIQQQQIIQQ", data, shoff + i * shentsize)
    stro = sh(shstrndx)[4]
    for i in range(shnum):
        h = sh(i)
        nm = data[stro + h[0]:data.index(b"\0", stro + h[0])].decode()
        if nm == name:
            return data[h[4]:h[4] + h[5]]
    raise ValueError(f"{path}: no section {name}")


def code_objects(path, arch="gfx950"):
    """Every `arch` code object in the library's offload bundles (one bundle
    per translation unit, concatenated in .hip_fatbin)."""
    fat = _section(path, ".hip_fatbin")
    out = []
    pos = fat.find(BUNDLE_MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", fat, pos + 24)
        q = pos + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", fat, q)
            triple = fat[q + 24:q + 24 + tlen].decode()
            q += 24 + tlen
            if triple.endswith(arch) and size:
                out.append(fat[pos + off:pos + off + size])
        pos = fat.find(BUNDLE_MAGIC, q)
    return out


def disassemble(co_bytes):
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "co.elf")
        with open(p, "wb") as f:
            f.write(co_bytes)
        return subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", p],
                              check=True, capture_output=True, text=True).stdout


def kernels(asm):
    """{symbol: body} per function of an llvm-objdump listing."""
    out = {}
    for m in re.finditer(r"^[0-9a-f]+ <(\S+)>:\n(.*?)(?=^[0-9a-f]+ <|\Z)", asm, re.M | re.S):
        out[m.group(1)] = m.group(2)
    return out


def audit(path=LIB):
    stats = {}
    bad = []
    spills = []
    ncos = 0
    for co in code_objects(path):
        ncos += 1
        for name, body in kernels(disassemble(co)).items():
            nsp = len(SPILL_RE.findall(body))
            if nsp:
                spills.append({"kernel": name, "scratch_ops": nsp})
            # Itanium mangling prefixes every name with its length: 9BF16Exact, 8F16Exact
            key = next((k for k in POLICIES if f"{len(k)}{k}" in name), None)
            if key is None:
                continue
            e = stats.setdefault(key, {"kernels": 0, "fma": 0, "mix": 0})
            e["kernels"] += 1
            fma = len(FMA_RE.findall(body))
            mix = len(MIX_RE.findall(body))
            e["fma"] += fma
            e["mix"] += mix
            if key in EXACT_KEYS and (fma or mix):
                bad.append({"kernel": name, "fma": fma, "mix": mix})
    return {"target": "gfx950", "library": os.path.relpath(path, ROOT), "code_objects": ncos, "per_policy": stats,
            "exact_policies_clean": not bad, "offending_kernels": bad, "spilling_kernels": spills}


def main():
    r = audit(sys.argv[1] if len(sys.argv) > 1 else LIB)
    print(json.dumps(r, indent=1))
    sys.exit(0 if r["exact_policies_clean"] else 1)


if __name__ == "__main__":
    main()
