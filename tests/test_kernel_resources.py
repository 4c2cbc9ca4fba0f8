"""Register budget of the hot kernels (CPU, hipcc cross-compile for gfx950): the bench kernels must not
spill VGPRs to scratch.  Round 2 found a silent 20 % regression of k_rollout when a new kernel in the
same translation unit changed the inliner's decision for attack_big (a real call, 60 spilled VGPRs,
288 B of scratch per lane and ~1.6 KB of extra HBM writes per agent-step)."""
import os
import re
import shutil
import subprocess

import pytest

import common

HOT = {
    "k_rollout<Battle, prefetch>": "_ZN3mfx9k_rolloutILb1ELb1ELb0E",
    "k_observe_items": "_ZN3mfx15k_observe_items",
    "k_rollout_big": "_ZN3mfx13k_rollout_big",
}


def _usage():
    hipcc = "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("hipcc not available")
    src = os.path.join(common.PKG, "csrc", "battle_kernels.hip")
    out = subprocess.run([hipcc, "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
                          "-mllvm", "-amdgpu-atomic-optimizer-strategy=None", "--cuda-device-only", "-c", "-x",
                          "hip", src, "-o", os.devnull, "-Rpass-analysis=kernel-resource-usage"],
                         capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-2000:]
    usage, cur = {}, None
    for line in out.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            usage[cur] = {}
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[bytes/lane\])?: (\d+)", line)
        if m and cur:
            usage[cur][m.group(1).strip()] = int(m.group(2))
    return usage


def test_hot_kernels_do_not_spill():
    usage = _usage()
    for name, prefix in HOT.items():
        hits = [k for k in usage if k.startswith(prefix)]
        assert hits, name
        for k in hits:
            u = usage[k]
            assert u.get("VGPRs Spill", 0) == 0, (name, u)
            assert u.get("ScratchSize", 0) == 0, (name, u)


def test_queue_kernel_register_budget():
    """k_rollout_bigq (the large-env bench kernel) inlines the step into the item loop: two 512-lane
    workgroups per CU (4 waves per SIMD, <= 128 VGPRs) with a few spills inside the step (72 B of
    scratch per lane).  The step as a real call needed 436 B of stack per lane and ran 11 % slower
    (profiles/r02_bigq_sweeps.txt); this bounds both."""
    usage = _usage()
    hits = [k for k in usage if k.startswith("_ZN3mfx14k_rollout_bigq")]
    assert hits
    for k in hits:
        u = usage[k]
        assert u.get("VGPRs", 999) <= 128, u
        assert u.get("ScratchSize", 0) <= 96, u
