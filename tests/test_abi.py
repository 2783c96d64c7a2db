"""The C ABI library loads and exports exactly what include/mpvae_hip.h declares
(no GPU needed: only host-side entry points are called)."""
import ctypes
import os
import re
import subprocess

import pytest

import mpvae_hip as H

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "mpvae_hip.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(mpv_[a-z0-9_]+)\s*\(", src)) - {"mpv_shape"})


def test_header_declares_the_binding_table():
    assert declared_functions() == sorted(H.SIGNATURES)


def test_library_exports_every_declared_symbol():
    lib = H.load_library()
    for name in declared_functions():
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", H.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (mpv_\w+)", out))
    assert exported == set(declared_functions())


def test_abi_version_and_host_entry_points():
    lib = H.load_library()
    assert lib.mpv_abi_version() == H.ABI_VERSION
    s = H.Shape(4096, 4096, 0, 512, 1024, 1024)
    fw, bw = lib.mpv_fwd_workspace_bytes(s), lib.mpv_bwd_workspace_bytes(s, H.GEMM_F32)
    assert 0 < fw < 1 << 30 and 0 < bw < 1 << 30
    # 3xf16: + the two fp16 planes of G (2 x 2 B x B*S x L)
    bw16 = lib.mpv_bwd_workspace_bytes(s, H.GEMM_F16X3)
    assert bw16 > bw and bw16 >= 4 * 512 * 4096 * 1024  # + the G hi/lo planes
    # invalid shapes are rejected on the host, before any launch
    bad = H.Shape(0, 10, 0, 4, 8, 8)
    assert lib.mpv_fwd_workspace_bytes(bad) == 0
    args = H.FwdArgs()
    assert lib.mpv_probit_fwd(bad, args, None) == 1
    assert b"sample range" in lib.mpv_last_error()
    assert lib.mpv_probit_fwd(H.Shape(4, 4, 0, 2, 8, 8), args, None) == 1
    assert b"NULL" in lib.mpv_last_error()
    assert lib.mpv_convert(None, 0, None, 0, 4, None) == 1


@pytest.mark.parametrize("L,z,cols", [(38, 38, 64), (64, 64, 64), (65, 38, 128), (38, 65, 128),
                                      (128, 5, 128), (2, 128, 128), (129, 5, 256),
                                      (5, 129, 256), (1024, 1024, 1024), (100, 300, 512)])
def test_noise_plane_cols_follow_the_dr_tile(L, z, cols):
    """Noise planes are padded to whole dR tiles: 64 columns when L and z are
    both <= 64, 128 when both are <= 128 (the 64 / 128 square tiles), else 256
    (probit_bwd.hip, dr16_tile)."""
    lib = H.load_library()
    assert lib.mpv_noise_plane_cols(H.Shape(16, 16, 0, 2, L, z)) == cols
    assert lib.mpv_noise_plane_cols(H.Shape(0, 16, 0, 2, L, z)) == 0  # bad shape


def test_check_raises_with_message():
    with pytest.raises(H.MPVError, match="NULL"):
        H.check(H.load_library().mpv_probit_bwd(H.Shape(4, 4, 0, 2, 8, 8), H.BwdArgs(), None),
                "mpv_probit_bwd")


def test_compute_loss_dispatches_on_device():
    """CPU tensors go to the host C++ backend (mpvae_host.py, as the reference
    runs its small configurations on the CPU), never to the HIP library; a
    mix of devices is an error.  CUDA tensors (tests/test_gpu_*) run the HIP
    library and raise when it is missing (test_missing_library_fails_loudly)."""
    import torch
    import mpvae
    import mpvae_host
    cpu = torch.zeros(2, 3)
    assert isinstance(mpvae._backend_for((cpu, cpu)), mpvae_host.HostShardBackend)
    assert mpvae._backend_for((cpu, None)) is not None


def test_missing_library_fails_loudly(tmp_path):
    with pytest.raises(H.MPVError, match="not found"):
        H.load_library(str(tmp_path / "nope.so"))


def test_linear_host_checks():
    """mpv_linear's workspace sizing and argument checks run on the host and
    reject bad problems before any launch (csrc/linear.hip)."""
    lib = H.load_library()
    assert lib.mpv_linear_workspace_bytes(0, 4, 4) == 0
    assert lib.mpv_linear_workspace_bytes(128, 256, 1000) > 0  # split-K partials
    fake = ctypes.c_void_p(0x1000)  # never dereferenced: every call below fails its checks
    ok = H.LinearArgs(M=4, N=4, R=4, a=fake, a_si=4, a_sr=1, b=fake, b_sj=4, b_sr=1, ones_col=-1,
                      alpha=1.0, out=fake, out_si=4)
    arr = (H.LinearArgs * 5)(ok, ok, ok, ok, ok)
    assert lib.mpv_linear_batch(arr, 5, None, 0, None) == 1  # at most 4 problems per launch
    assert b"problems per launch" in lib.mpv_last_error()
    assert lib.mpv_linear_batch(arr, 0, None, 0, None) == 1
    no_out = H.LinearArgs(M=4, N=4, R=4, a=fake, b=fake, ones_col=-1, alpha=1.0)
    assert lib.mpv_linear(ctypes.byref(no_out), None, 0, None) == 1
    bad_ones = H.LinearArgs(M=4, N=4, R=4, a=fake, a_si=4, a_sr=1, b=fake, b_sj=4, b_sr=1,
                            ones_col=1, alpha=1.0, out=fake, out_si=4)
    assert lib.mpv_linear(ctypes.byref(bad_ones), None, 0, None) == 1
    big = H.LinearArgs(M=128, N=256, R=1000, a=fake, a_si=1000, a_sr=1, b=fake, b_sj=1000,
                       b_sr=1, ones_col=-1, alpha=1.0, out=fake, out_si=256)
    assert lib.mpv_linear(ctypes.byref(big), None, 0, None) == 1  # no workspace for the partials
    assert b"workspace" in lib.mpv_last_error()
    # a second reduction segment needs both operands and no mask (ABI v8)
    half = H.LinearArgs(M=4, N=4, R=4, a=fake, a_si=4, a_sr=1, b=fake, b_sj=4, b_sr=1,
                        ones_col=-1, alpha=1.0, out=fake, out_si=4, a2=fake, a2_si=4, R1=2)
    assert lib.mpv_linear(ctypes.byref(half), None, 0, None) == 1
    assert b"second segment" in lib.mpv_last_error()


HOST_HEADER = os.path.join(ROOT, "include", "mpvae_host.h")


def test_host_library_exports_what_its_header_declares():
    """libmpvae_host.so (the CPU backend) against include/mpvae_host.h."""
    import mpvae_host
    src = re.sub(r"/\*.*?\*/", "", open(HOST_HEADER).read(), flags=re.S)
    declared = sorted(set(re.findall(r"\b(mpvh_[a-z0-9_]+)\s*\(", src)))
    assert declared == mpvae_host.EXPORTS
    lib = mpvae_host.load_library()
    assert lib.mpvh_abi_version() == mpvae_host.ABI_VERSION
    out = subprocess.run(["nm", "-D", "--defined-only", mpvae_host.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    assert set(re.findall(r"\bT (mpvh_\w+)", out)) == set(declared)
    assert lib.mpvh_probit_fwd(H.Shape(0, 4, 0, 2, 8, 8), mpvae_host.FwdArgs()) == 1
    assert b"bad shape" in lib.mpvh_last_error()
