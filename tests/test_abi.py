"""libsvgpu.so C ABI: loads, exports every prototype in include/svgpu.h, argument/emptiness errors
without compute, loud failure without a GPU, and the host-only fold."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT
from oracle import bn254 as b


def _header_functions():
    src = open(os.path.join(ROOT, "include", "svgpu.h")).read()
    return sorted(set(re.findall(r"\b(sv_[a-z0-9_]+)\s*\(", src)))


def test_library_loads_and_exports_every_header_symbol():
    import svgpu
    from svgpu import _lib
    names = _header_functions()
    assert len(names) >= 13
    for n in names:
        assert hasattr(_lib.lib, n), f"{n} declared in svgpu.h but not exported"
    assert {p[0] for p in _lib.PROTOTYPES} == set(names), "ctypes prototypes out of sync with svgpu.h"
    assert "gfx950" in svgpu.version()


def test_struct_layouts_match_header():
    from svgpu import _lib
    assert ctypes.sizeof(_lib.sv_fe) == 32
    assert ctypes.sizeof(_lib.sv_g1_affine) == 64
    assert ctypes.sizeof(_lib.sv_g1_jacobian) == 96
    assert ctypes.sizeof(_lib.sv_g2_affine) == 128
    assert ctypes.sizeof(_lib.sv_fq12) == 384


def test_empty_inputs_map_to_reference_panics():
    import svgpu
    with pytest.raises(svgpu.ReferencePanic, match="pairs should not be empty"):
        svgpu.NativeLoader.multi_scalar_multiplication([])
    with pytest.raises(svgpu.ReferencePanic):
        svgpu.KzgAs.decide_all(svgpu.KzgDecidingKey(b.G1_GEN, b.G2_GEN, b.G2_GEN), [])
    from svgpu import _lib
    out = _lib.sv_g1_affine()
    assert _lib.lib.sv_bn254_g1_msm(None, None, 0, 0, 0, ctypes.byref(out)) == _lib.SV_ERR_EMPTY
    assert "empty" in _lib.last_error()


def test_bad_arguments_rejected():
    from svgpu import _lib
    out = _lib.sv_g1_affine()
    buf = np.zeros(16, np.uint64)
    assert _lib.lib.sv_bn254_g1_msm(buf.ctypes.data, buf.ctypes.data, 1, 7, 0, ctypes.byref(out)) == _lib.SV_ERR_ARG
    assert _lib.lib.sv_bn254_g1_msm(None, buf.ctypes.data, 1, 0, 0, ctypes.byref(out)) == _lib.SV_ERR_ARG


def test_fold_is_host_only_and_exact():
    import svgpu
    pts = [b.g1_mul(b.G1_GEN, k) for k in (3, 5, 7, 11)]
    z = [2, 3, 1, 5]
    parts = [(x * zz * zz % b.P, y * zz**3 % b.P, zz) for (x, y), zz in zip(pts, z)]
    assert svgpu.fold_partials(parts) == b.g1_mul(b.G1_GEN, 26)
    assert svgpu.fold_partials([(1, 1, 0)]) is None
    assert svgpu.fold_partials(parts + [(pts[0][0], (-pts[0][1]) % b.P, 1)]) == b.g1_mul(b.G1_GEN, 23)
    with pytest.raises(svgpu.ArgumentError):
        svgpu.fold_partials([(b.P, 1, 1)])


def _has_gpu():
    import torch
    return torch.cuda.is_available()


@pytest.mark.skipif(_has_gpu(), reason="checks the no-GPU behaviour")
def test_compute_without_gpu_fails_loudly():
    import svgpu
    with pytest.raises(svgpu.DeviceError):
        svgpu.multi_scalar_multiplication([1], [b.G1_GEN])


def test_poseidon_arguments_rejected_without_compute():
    from svgpu import _lib, poseidon as gp
    buf = np.zeros(16, np.uint64)
    off = np.zeros(2, np.uint64)
    assert _lib.lib.sv_bn254_poseidon_permute(buf.ctypes.data, 1, 4, 0) == _lib.SV_ERR_ARG
    assert _lib.lib.sv_bn254_poseidon_permute(buf.ctypes.data, 1, 3, 9) == _lib.SV_ERR_ARG
    assert _lib.lib.sv_bn254_poseidon_permute(buf.ctypes.data, 0, 3, 0) == _lib.SV_OK  # nothing to do
    bad = np.array([2, 1], np.uint64)
    assert _lib.lib.sv_bn254_poseidon_squeeze(buf.ctypes.data, buf.ctypes.data, bad.ctypes.data, 1, 3, 0,
                                              None) == _lib.SV_ERR_ARG
    assert _lib.lib.sv_bn254_poseidon_squeeze(None, buf.ctypes.data, off.ctypes.data, 1, 3, 0,
                                              None) == _lib.SV_ERR_ARG
    with pytest.raises(_lib.ArgumentError):
        gp.Poseidon(4)
    with pytest.raises(_lib.LengthError):
        gp.permute([[1, 2]], 3)
    assert gp.permute([], 3) == [] and gp.squeeze_many([]) == []


def test_msm_batch_arguments_rejected_without_compute():
    import svgpu
    from svgpu import _lib
    buf = np.zeros(64, np.uint64)
    out = np.zeros(64, np.uint64)
    bad = np.array([0, 2, 1], np.uint64)
    assert _lib.lib.sv_bn254_g1_msm_batch(buf.ctypes.data, buf.ctypes.data, bad.ctypes.data, 2, 0,
                                          out.ctypes.data) == _lib.SV_ERR_ARG
    empty = np.array([0, 1, 1], np.uint64)
    assert _lib.lib.sv_bn254_g1_msm_batch(buf.ctypes.data, buf.ctypes.data, empty.ctypes.data, 2, 0,
                                          out.ctypes.data) == _lib.SV_ERR_EMPTY
    assert _lib.lib.sv_bn254_g1_msm_batch(None, None, None, 0, 0, None) == _lib.SV_OK
    with pytest.raises(svgpu.ReferencePanic, match="pairs should not be empty"):
        svgpu.batch_multi_scalar_multiplication([[(1, b.G1_GEN)], []])
    assert svgpu.batch_multi_scalar_multiplication([]) == []


def test_base_table_arguments_rejected_without_compute():
    from svgpu import _lib
    buf = np.zeros(64, np.uint64)
    h = ctypes.c_uint64(0)
    assert _lib.lib.sv_bn254_g1_table_create(buf.ctypes.data, 0, 0, 0, ctypes.byref(h)) == _lib.SV_ERR_EMPTY
    assert _lib.lib.sv_bn254_g1_table_create(buf.ctypes.data, 1, 9, 0, ctypes.byref(h)) == _lib.SV_ERR_ARG
    assert _lib.lib.sv_bn254_g1_table_create(None, 1, 0, 0, ctypes.byref(h)) == _lib.SV_ERR_ARG
    assert _lib.lib.sv_bn254_g1_table_destroy(123456789) == _lib.SV_ERR_ARG
    assert "unknown base table" in _lib.last_error()
    idx = np.zeros(4, np.uint32)
    bad = np.array([0, 2, 1], np.uint64)
    empty = np.array([0, 1, 1], np.uint64)
    good = np.array([0, 1, 2], np.uint64)
    out = np.zeros(64, np.uint64)
    call = _lib.lib.sv_bn254_g1_msm_batch_table
    assert call(1, idx.ctypes.data, buf.ctypes.data, bad.ctypes.data, 2, 0, out.ctypes.data) == _lib.SV_ERR_ARG
    assert call(1, idx.ctypes.data, buf.ctypes.data, empty.ctypes.data, 2, 0, out.ctypes.data) == _lib.SV_ERR_EMPTY
    assert call(987654, idx.ctypes.data, buf.ctypes.data, good.ctypes.data, 2, 0, out.ctypes.data) == _lib.SV_ERR_ARG
    assert call(1, None, None, None, 0, 0, None) == _lib.SV_OK
    dev = _lib.lib.sv_bn254_g1_msm_batch_indexed_device
    assert dev(buf.ctypes.data, 0, 0, idx.ctypes.data, buf.ctypes.data, good.ctypes.data, 2, 1, 0, 0, None,
               out.ctypes.data) == _lib.SV_ERR_EMPTY


def test_codec_arguments_rejected_without_compute():
    from svgpu import _lib
    buf = np.zeros(64, np.uint8)
    out = np.zeros(16, np.uint64)
    bad = ctypes.c_int64(5)
    assert _lib.lib.sv_bn254_g1_decode(buf.ctypes.data, 1, 7, 0, out.ctypes.data, ctypes.byref(bad)) == _lib.SV_ERR_ARG
    assert _lib.lib.sv_bn254_g1_decode(buf.ctypes.data, 0, 0, 0, out.ctypes.data, ctypes.byref(bad)) == _lib.SV_OK
    assert bad.value == -1
    ff = ctypes.c_int32(0)
    assert _lib.lib.sv_bn254_kzg_decide_eip197(buf.ctypes.data, 0, 0, ctypes.byref(ff)) == _lib.SV_ERR_EMPTY
    recs = np.zeros(2 * 0x180, np.uint8)
    recs[0x180 + 64] = 1  # record 1 carries a different G2 than record 0
    assert _lib.lib.sv_bn254_kzg_decide_eip197(recs.ctypes.data, 2, 0, ctypes.byref(ff)) == _lib.SV_ERR_ARG
    assert "differ" in _lib.last_error()


def test_accumulate_rejects_unreduced_r_without_compute():
    """sv_bn254_kzg_accumulate validates r < the Fr order on the host, like every other scalar input."""
    from svgpu import _lib
    from svgpu import encoding as enc
    pts = enc.bases_array([b.G1_GEN])
    out_l, out_r = _lib.sv_g1_affine(), _lib.sv_g1_affine()
    for bad in (b.R, b.R + 5, (1 << 256) - 1):
        rr = _lib.sv_fe()
        for i in range(4):
            rr.l[i] = (bad >> (64 * i)) & ((1 << 64) - 1)
        rc = _lib.lib.sv_bn254_kzg_accumulate(pts.ctypes.data, pts.ctypes.data, 1, ctypes.byref(rr), 0, 0,
                                              ctypes.byref(out_l), ctypes.byref(out_r))
        assert rc == _lib.SV_ERR_ARG, bad
        assert "not reduced" in _lib.last_error()


def test_library_stamp_matches_sources():
    """build/libsvgpu.so was linked from the sources in this tree (build/SOURCES.sha256, written by
    the Makefile; svgpu/_lib.py refuses a stale library at import, so a prebuilt .so that travels to
    the GPU box with changed sources fails loudly instead of testing old code)."""
    import os
    from svgpu import _lib, _srchash
    stamp = os.path.join(os.path.dirname(_lib.LIB_PATH), "SOURCES.sha256")
    assert open(stamp).read().strip() == _srchash.source_hash()
    assert any(p.endswith("msm.hip") for p in _srchash.source_files())
