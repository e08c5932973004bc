"""Exactness guard at build time: the gfx950 ISA of every
exact-policy kernel in the BUILT libdlsim_hip.so has no fused multiply-add and
no mixed-precision instruction. The reference rounds every product and every
sum separately (fedavg.py:25), so a launch-shape change that
lets the backend contract `acc + w*x` fails this CPU test before any GPU run.
"""
from __future__ import annotations

import json
import os
import re
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "scripts"))
import audit_isa  # noqa: E402


@pytest.fixture(scope="module")
def report():
    if not os.path.exists(audit_isa.LIB):
        pytest.fail("libdlsim_hip.so is not built (run __graft_entry__.build())")
    return audit_isa.audit()


def test_every_translation_unit_with_device_code_is_audited(report):
    # one code object per inst_*.hip unit, plus sharded_abi.hip's unpad copy
    # kernel and dlsim_abi.hip's mixed-dtype fold (round 5)
    units = [f for f in os.listdir(os.path.join(ROOT, "decentralized-learning-simulator_amd", "csrc"))
             if f.startswith("inst_") and f.endswith(".hip")]
    assert report["code_objects"] == len(units) + 2


def test_exact_kernels_have_no_fused_or_mixed_ops(report):
    assert report["exact_policies_clean"], json.dumps(report["offending_kernels"][:10], indent=1)
    for pol in ("F32Exact", "BF16Exact", "F16Exact", "F64Exact"):
        assert report["per_policy"][pol]["kernels"] > 40, pol
    assert report["per_policy"]["MixedSlots"]["kernels"] == 1  # k_wreduce_mixed, audited as exact


def test_audit_sees_the_round2_shapes():
    """The fixed VPT-2 block-map and grouped VPT-1 wave-map shapes
    (dispatch.hpp fixed_shape / grouped_shape) are among the audited kernels."""
    names = set()
    for co in audit_isa.code_objects(audit_isa.LIB):
        names |= set(audit_isa.kernels(audit_isa.disassemble(co)))
    exact = [n for n in names if "8F32Exact" in n and "k_wreduce_tiles" in n]
    # template args <Op, S, NF, G, VPT, NT, STP, WAVE>: ...ELi<VPT>ELi1ELi<STP>ELb<wave>E,
    # STP = 2 (buffer store, nt; round 5)
    assert any("ELi2ELi1ELi2ELb0E" in n for n in exact), "fixed VPT 2 block map missing"
    assert any("ELi0ELi8ELi1ELi1ELi2ELb1E" in n for n in exact), "grouped VPT 1 wave map missing"
    assert any("ELi4ELi1ELi2ELb1E" in n for n in exact), "VPT 4 wave map missing"


def test_detector_catches_contraction(report):
    # positive controls: the FAST policies fuse by design, and the patterns
    # match the instructions a contraction would produce
    assert report["per_policy"]["F32Fast"]["fma"] > 0
    assert report["per_policy"]["F64Fast"]["fma"] > 0
    for ins in ("v_fma_f32 v1, v2, v3, v4", "v_fmac_f32_e32 v1, v2, v3", "v_pk_fma_f32 v[0:1], v[2:3], v[4:5], v[6:7]",
                "v_fma_f64 v[0:1], v[2:3], v[4:5], v[6:7]"):
        assert audit_isa.FMA_RE.search(ins), ins
    assert audit_isa.MIX_RE.search("v_fma_mixlo_f16 v1, v2, v3, v4")


def test_no_kernel_spills_and_deferred_kernels_present(report):
    """No kernel of the library spills registers to scratch (the deferred-store
    kernel keeps up to 32 results per lane in VGPRs: a rolled loop would put
    them in scratch, and its grouped form reads its kernel-argument slots in
    place), and the deferred kernels exist for fp32 fixed fan-in 4..14 and the
    grouped form, instantiated from fan-in 2 (dispatch.hpp defer_eligible,
    DESIGN.md §5e)."""
    assert report["spilling_kernels"] == [], json.dumps(report["spilling_kernels"][:10], indent=1)
    names = set()
    for co in audit_isa.code_objects(audit_isa.LIB):
        names |= set(audit_isa.kernels(audit_isa.disassemble(co)))
    for pol in ("8F32Exact", "7F32Fast", "7F32Mean"):
        got = sorted(n for n in names if "k_wreduce_defer" in n and pol in n)
        # template args <Op, S, NF, G, RMAX, U, STP, RC>: ...ELi<NF>ELi8ELi<RMAX>ELi2ELi2ELi<RC>EE
        # (RMAX 24 from NF 12; NF 0 = the grouped form; RC 0 = runtime R)
        for nf in list(range(2, 15)) + [0]:
            assert any(f"ELi{nf}ELi8ELi{32 if nf < 12 else 24}ELi2ELi2ELi0EE" in n for n in got), (pol, nf)
        assert not any(f"ELi1ELi8ELi32ELi2ELi2ELi0EE" in n for n in got), pol
    # the exact policy's fixed fan-in kernels compiled per even R (dispatch.hpp
    # launch_defer_rc): from R = 4 (defer_rows' least) for fan-in 3-14 (the
    # default deferral floor is fan-in 3); R = 2 and fan-in 2 (reachable only
    # through the A/B switches) take the runtime R. Round 6: 168 compiled-R
    # kernels (round 5: 196, fan-in 2 and R = 2 included).
    exact = [n for n in names if "k_wreduce_defer" in n and "8F32Exact" in n]
    by_nf = {}
    for n in exact:
        m = re.search(r"EELi(\d+)ELi8ELi(\d+)ELi2ELi2ELi(\d+)EE", n)
        if m and int(m.group(3)) > 0:
            by_nf.setdefault(int(m.group(1)), set()).add((int(m.group(2)), int(m.group(3))))
    assert sorted(by_nf) == list(range(3, 15)), sorted(by_nf)
    for nf, got in by_nf.items():
        rmax = 32 if nf < 12 else 24
        assert got == {(rmax, rc) for rc in range(4, rmax + 1, 2)}, (nf, sorted(got))
    assert sum(len(v) for v in by_nf.values()) == 168
