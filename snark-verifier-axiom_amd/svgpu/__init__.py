"""svgpu -- MI355X-native BN254 MSM + KZG decider behind snark-verifier's native hot-path API.

Mirrors (reference = yuliakot/snark-verifier-axiom):
  NativeLoader.multi_scalar_multiplication   snark-verifier/src/loader/native.rs:61-71
  multi_scalar_multiplication                snark-verifier/src/util/msm.rs:287-316
  KzgAs.decide / decide_all                  snark-verifier/src/pcs/kzg/decider.rs:60-80
  KzgAs.create_proof / verify (no blind)     snark-verifier/src/pcs/kzg/accumulation.rs:146-195
  Poseidon / PoseidonTranscript              snark-verifier/src/util/hash/poseidon.rs:412-467,
                                             system/halo2/transcript/halo2.rs:198-227
All compute runs in libsvgpu.so (HIP, gfx950); there is no CPU fallback.
"""
from ._lib import (SV_CANONICAL, SV_MONTGOMERY, ArgumentError, DeviceError, EmptyError, LengthError,
                   OutOfMemoryError, SvError, lib)
from .kzg import AssertionFailure, KzgAccumulator, KzgAs, KzgDecidingKey
from .loader import (BaseTable, NativeLoader, ReferencePanic, batch_multi_scalar_multiplication, fold_partials, msm_arrays,
                     make_refs, msm_batch_arrays, msm_refs, multi_scalar_multiplication)
from .poseidon import Poseidon, PoseidonTranscript


def init(num_devices: int = 0) -> int:
    from ._lib import check
    check(lib.sv_init(num_devices), "sv_init")
    return lib.sv_device_count()


def version() -> str:
    return lib.sv_version().decode()
