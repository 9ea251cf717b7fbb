"""The AQL engine writes kernel arguments itself (cksum_kernels.hip,
aql_fill_args / aql_fill_raw): the explicit arguments in parameter order,
then -- for kernels that read them -- the code-object-v5 hidden block counts,
group sizes, remainders and grid dimensions at fixed offsets.  This CPU test
reads the kernels' own metadata out of the built library's gfx950 code object
and checks that every mi_aql_* entry point has the layout the engine assumes
(no GPU needed)."""
import os
import re
import shutil
import subprocess

import pytest

from libunsod_amd._lib import LIB_PATH

LLVM = "/opt/rocm/llvm/bin"
BUNDLER = os.path.join(LLVM, "clang-offload-bundler")
READELF = os.path.join(LLVM, "llvm-readelf")

# the explicit arguments the engine writes: Desc (80 B) + ip, l4, st, bad
VERIFY_EXPLICIT = 112
SCALAR_EXPLICIT = 56  # mi_aql_scalar's 12 parameters
HIDDEN = {"hidden_block_count_x": 0, "hidden_block_count_y": 4, "hidden_block_count_z": 8,
          "hidden_group_size_x": 12, "hidden_group_size_y": 14, "hidden_group_size_z": 16,
          "hidden_remainder_x": 18, "hidden_remainder_y": 20, "hidden_remainder_z": 22,
          "hidden_global_offset_x": 40, "hidden_global_offset_y": 48, "hidden_global_offset_z": 56,
          "hidden_grid_dims": 64}


def _kernels(tmp_path):
    if not (os.path.exists(BUNDLER) and os.path.exists(READELF) and shutil.which("objcopy")):
        pytest.skip("LLVM / binutils tools not available")
    fat = tmp_path / "fatbin.bin"
    co = tmp_path / "co.elf"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", LIB_PATH, str(fat)], check=True)
    subprocess.run([BUNDLER, "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    notes = subprocess.run([READELF, "--notes", str(co)], check=True, capture_output=True, text=True).stdout
    out = {}
    # one YAML block per kernel: '.args:' ... '.name: <kernel>'
    for block in re.split(r"\n  - \.agpr_count:", notes):
        m = re.search(r"\.name:\s+(mi_aql_\w+)", block)
        if not m:
            continue
        args = re.findall(r"\.offset:\s+(\d+)\s+\.size:\s+(\d+)\s+\.value_kind:\s+(\w+)", block)
        seg = int(re.search(r"\.kernarg_segment_size:\s+(\d+)", block).group(1))
        out[m.group(1)] = ([(int(o), int(s), k) for o, s, k in args], seg)
    return out


def test_aql_entry_points_kernarg_layout(tmp_path):
    ks = _kernels(tmp_path)
    verify = [k for k in ks if k not in ("mi_aql_scalar", "mi_aql_dropin_svc", "mi_aql_spin", "mi_aql_tx_lds")]
    assert "mi_aql_v_16x6" in ks and "mi_aql_run8" in ks and "mi_aql_slot64" in ks and "mi_aql_scalar" in ks
    assert "mi_aql_vd_16x6" in ks and "mi_aql_vd_8x12" in ks and "mi_aql_tx_lds" in ks
    # mi_aql_tx_lds(TxDesc): one 120-byte by-value argument, the hidden block
    # right after it (aql_create_tx writes sizeof(TxDesc) bytes, then kAqlTxHidden)
    args, seg = ks["mi_aql_tx_lds"]
    explicit = [(o, s) for o, s, k in args if not k.startswith("hidden_")]
    assert explicit == [(0, 120)], explicit
    for o, s, k in args:
        if k in HIDDEN:
            assert o == 120 + HIDDEN[k], ("mi_aql_tx_lds", k, o)
    assert seg <= 512, seg
    for name in verify:
        args, seg = ks[name]
        explicit = [(o, s) for o, s, k in args if not k.startswith("hidden_")]
        # mi_aql_vd_*: one more argument, the queue's dealt-unit counter set (AqlDealArgs)
        deal = name.startswith("mi_aql_vd_")
        assert explicit == [(0, 80), (80, 8), (88, 8), (96, 8), (104, 8)] + ([(112, 8)] if deal else []), (name, explicit)
        for o, s, k in args:
            if k in HIDDEN:
                assert o == VERIFY_EXPLICIT + (8 if deal else 0) + HIDDEN[k], (name, k, o)
        assert seg <= 512, (name, seg)
    args, seg = ks["mi_aql_scalar"]
    explicit = [(o, s) for o, s, k in args if not k.startswith("hidden_")]
    assert explicit[0] == (0, 8) and explicit[-1] == (48, 8) and len(explicit) == 12, explicit
    # the engine writes hidden arguments only when the segment holds them
    if seg > SCALAR_EXPLICIT:
        for o, s, k in args:
            if k in HIDDEN:
                assert o == SCALAR_EXPLICIT + HIDDEN[k], ("mi_aql_scalar", k, o)
    # mi_aql_dropin_svc(slab, nslots, exitw, token, idle_ticks): SvcArgs in
    # svc_ensure, 32 bytes
    args, seg = ks["mi_aql_dropin_svc"]
    explicit = [(o, s) for o, s, k in args if not k.startswith("hidden_")]
    assert explicit == [(0, 8), (8, 4), (16, 8), (24, 4), (28, 4)], explicit
    if seg > 32:
        for o, s, k in args:
            if k in HIDDEN:
                assert o == 32 + HIDDEN[k], ("mi_aql_dropin_svc", k, o)


def _all_kernel_notes(tmp_path):
    if not (os.path.exists(BUNDLER) and os.path.exists(READELF) and shutil.which("objcopy")):
        pytest.skip("LLVM / binutils tools not available")
    fat = tmp_path / "fatbin_all.bin"
    co = tmp_path / "co_all.elf"
    subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", LIB_PATH, str(fat)], check=True)
    subprocess.run([BUNDLER, "--unbundle", "--type=o", f"--input={fat}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    notes = subprocess.run([READELF, "--notes", str(co)], check=True, capture_output=True, text=True).stdout
    out = {}
    for block in re.split(r"\n  - \.agpr_count:", notes)[1:]:
        name = re.search(r"\.name:\s+(\S+)", block).group(1)
        priv = int(re.search(r"\.private_segment_fixed_size:\s+(\d+)", block).group(1))
        dyn = re.search(r"\.uses_dynamic_stack:\s+(\w+)", block).group(1)
        out[name] = (priv, dyn)
    return out


def test_no_kernel_uses_scratch(tmp_path):
    """Every kernel of the library runs without a private segment (scratch).
    Round 2's k_ipv4_finalize<BLOCKS> kept its deferred-store state in a
    12-byte stack object (a pointer select the optimiser made from stores in
    two branches) and was the only kernel with scratch -- and the one that hit
    hipErrorIllegalAddress in the driver's suite.  A kernel that picks up
    scratch again (a dynamically indexed array, an address-taken local) fails
    here, on the CPU, before it reaches a GPU."""
    ks = _all_kernel_notes(tmp_path)
    assert len(ks) > 100, len(ks)
    assert any("k_ipv4_finalize" in k for k in ks)
    bad = {k: v for k, v in ks.items() if v != (0, "false")}
    assert not bad, bad
