"""Host-side encodings between Python ints / points and the C-ABI layouts.

Layouts (include/svgpu.h): an element is 4 x u64 little-endian limbs, canonical or Montgomery
(R = 2^256); a G1 affine point is x || y (64 B) with identity (0, 0); G2 affine is
x.c0 || x.c1 || y.c0 || y.c1 (128 B).  Points are Python tuples (x, y) of canonical ints, G2
coordinates are ((x0, x1), (y0, y1)); None is the identity.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib

P = 21888242871839275222246405745257275088696311157297823662689037894645226208583
R = 21888242871839275222246405745257275088548364400416034343698204186575808495617
_MASK256 = (1 << 256) - 1
_ZERO64 = bytes(64)


def _to_form(x: int, mod: int, form: int) -> int:
    return (x << 256) % mod if form == _lib.SV_MONTGOMERY else x


def _from_form(x: int, mod: int, form: int) -> int:
    return x * pow(1 << 256, -1, mod) % mod if form == _lib.SV_MONTGOMERY else x


def ints_to_limbs(values: Sequence[int]) -> np.ndarray:
    """(n,) ints < 2^256 -> (n, 4) uint64 little-endian limbs."""
    buf = b"".join(int(v).to_bytes(32, "little") for v in values)
    return np.frombuffer(buf, dtype=np.uint64).reshape(len(values), 4).copy()


def limbs_to_int(limbs) -> int:
    a = np.asarray(limbs, dtype=np.uint64)
    return int.from_bytes(a.tobytes(), "little")


def scalars_array(scalars: Sequence[int], form: int = _lib.SV_CANONICAL) -> np.ndarray:
    for s in scalars:
        if not 0 <= s < R:
            raise ValueError("scalar must be a reduced Fr element (0 <= s < r)")
    return ints_to_limbs([_to_form(s, R, form) for s in scalars])


def bases_array(points: Sequence[Optional[Tuple[int, int]]], form: int = _lib.SV_CANONICAL) -> np.ndarray:
    if form == _lib.SV_CANONICAL:  # one bytes join (2x faster than the generic path: config 5's encode)
        buf = b"".join(_ZERO64 if pt is None else (pt[0] % P).to_bytes(32, "little") + (pt[1] % P).to_bytes(32, "little")
                       for pt in points)
        return np.frombuffer(buf, dtype=np.uint64).reshape(len(points), 8).copy()
    flat: List[int] = []
    for pt in points:
        if pt is None:
            flat += [0, 0]
        else:
            flat += [_to_form(pt[0] % P, P, form), _to_form(pt[1] % P, P, form)]
    return ints_to_limbs(flat).reshape(len(points), 8)


def g1_from_struct(a: _lib.sv_g1_affine, form: int = _lib.SV_CANONICAL):
    x = limbs_to_int(list(a.x.l))
    y = limbs_to_int(list(a.y.l))
    if x == 0 and y == 0:
        return None
    return (_from_form(x, P, form), _from_form(y, P, form))


def g1_from_limbs(row, form: int = _lib.SV_CANONICAL):
    row = np.asarray(row, dtype=np.uint64)
    x, y = limbs_to_int(row[:4]), limbs_to_int(row[4:8])
    if x == 0 and y == 0:
        return None
    return (_from_form(x, P, form), _from_form(y, P, form))


def fe_struct(x: int) -> _lib.sv_fe:
    s = _lib.sv_fe()
    for i in range(4):
        s.l[i] = (x >> (64 * i)) & 0xFFFFFFFFFFFFFFFF
    return s


def g1_struct(pt, form: int = _lib.SV_CANONICAL) -> _lib.sv_g1_affine:
    s = _lib.sv_g1_affine()
    if pt is not None:
        s.x = fe_struct(_to_form(pt[0], P, form))
        s.y = fe_struct(_to_form(pt[1], P, form))
    return s


def g2_struct(q, form: int = _lib.SV_CANONICAL) -> _lib.sv_g2_affine:
    s = _lib.sv_g2_affine()
    if q is not None:
        (x0, x1), (y0, y1) = q
        s.x.c0, s.x.c1 = fe_struct(_to_form(x0, P, form)), fe_struct(_to_form(x1, P, form))
        s.y.c0, s.y.c1 = fe_struct(_to_form(y0, P, form)), fe_struct(_to_form(y1, P, form))
    return s


def jacobian_from_struct(j: _lib.sv_g1_jacobian) -> Tuple[int, int, int]:
    return (limbs_to_int(list(j.x.l)), limbs_to_int(list(j.y.l)), limbs_to_int(list(j.z.l)))


def jacobian_struct(X: int, Y: int, Z: int) -> _lib.sv_g1_jacobian:
    s = _lib.sv_g1_jacobian()
    s.x, s.y, s.z = fe_struct(X), fe_struct(Y), fe_struct(Z)
    return s


def fq12_from_struct(g: _lib.sv_fq12) -> List[int]:
    out = []
    for k in range(6):
        out.append(limbs_to_int(list(g.c[k].c0.l)))
        out.append(limbs_to_int(list(g.c[k].c1.l)))
    return out
