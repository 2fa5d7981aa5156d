"""Host-side encodings of the reference interface mirror (no GPU)."""
import numpy as np
import pytest

from oracle import bn254 as b


def test_roundtrip_forms():
    from svgpu import encoding as enc, SV_CANONICAL, SV_MONTGOMERY
    pts = [b.G1_GEN, None, b.g1_mul(b.G1_GEN, 77)]
    for form in (SV_CANONICAL, SV_MONTGOMERY):
        arr = enc.bases_array(pts, form)
        assert arr.shape == (3, 8)
        assert [enc.g1_from_limbs(r, form) for r in arr] == pts
    assert (enc.bases_array([None])[0] == 0).all()
    m = enc.bases_array([b.G1_GEN], SV_MONTGOMERY)[0]
    assert enc.limbs_to_int(m[:4]) == b.to_mont(1)


def test_scalar_validation():
    from svgpu import encoding as enc
    with pytest.raises(ValueError):
        enc.scalars_array([b.R])
    a = enc.scalars_array([0, 1, b.R - 1])
    assert [enc.limbs_to_int(r) for r in a] == [0, 1, b.R - 1]


def test_halo2curves_layout_is_little_endian_u64_limbs():
    from svgpu import encoding as enc
    x = 0x0102030405060708_1112131415161718_2122232425262728_3132333435363738
    row = enc.ints_to_limbs([x])[0]
    assert row[0] == 0x3132333435363738 and row[3] == 0x0102030405060708


def test_length_mismatch_panics():
    import svgpu
    with pytest.raises(svgpu.ReferencePanic):
        svgpu.multi_scalar_multiplication([1, 2], [b.G1_GEN])


def test_g2_cache_key_accepts_nested_lists():
    """A G2 point given as nested lists (accepted by enc.g2_struct) keys the per-key struct cache
    too (an unhashable list key broke decide())."""
    from svgpu import device as dv
    from oracle import bn254 as b
    q = b.G2_GEN
    as_lists = [[q[0][0], q[0][1]], [q[1][0], q[1][1]]]
    a = dv._g2_struct_cached(as_lists, 0)
    c = dv._g2_struct_cached(q, 0)
    assert bytes(a) == bytes(c)
    assert dv._g2_struct_cached(as_lists, 0) is a or bytes(dv._g2_struct_cached(as_lists, 0)) == bytes(a)


def test_g2_cache_identity_fast_path_sees_mutation():
    """The identity-keyed fast path (the same key object passed again) returns the cached struct only
    while the object's contents are unchanged: a list mutated in place gets the new point's struct."""
    from svgpu import device as dv
    from svgpu import encoding as enc
    from oracle import bn254 as b
    q, s = b.G2_GEN, b.g2_mul(b.G2_GEN, 5)
    key = [[q[0][0], q[0][1]], [q[1][0], q[1][1]]]
    first = dv._g2_struct_cached(key, 0)
    assert dv._g2_struct_cached(key, 0) is first
    key[0][0], key[0][1], key[1][0], key[1][1] = s[0][0], s[0][1], s[1][0], s[1][1]
    assert bytes(dv._g2_struct_cached(key, 0)) == bytes(enc.g2_struct(s, 0))
    arr = [list(map(int, c)) for c in q]
    assert bytes(dv._g2_struct_cached(arr, 1)) == bytes(enc.g2_struct(arr, 1))
