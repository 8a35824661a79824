"""ctypes binding of libinsr_hip.so (C ABI declared in include/insr_siren.h).

The library is the product: there is no CPU or eager-torch fallback behind it.
If it is missing or was not built, every hot-path call raises NativeUnavailable.
torch is imported first so the library binds to the HIP runtime torch already
loaded (both carry SONAME libamdhip64.so.7).
"""
import contextlib
import ctypes
import os
import threading

import torch  # noqa: F401  (must precede the CDLL load: shared HIP runtime)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("INSR_HIP_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libinsr_hip.so"))

MODE_VALUE, MODE_GRAD, MODE_LAP = 0, 1, 2
MODE_MASK, MODE_PREC_SHIFT = 0xF, 4
MODE_WSPLIT = 1 << 8  # the params buffer carries up-to-date pre-split weight planes
PREC_F32, PREC_BF16X6, PREC_BF16X3, PREC_BF16, PREC_F16X3 = 0, 1, 2, 3, 4
PRECISIONS = {"fp32": PREC_F32, "bf16x6": PREC_BF16X6, "bf16x3": PREC_BF16X3, "bf16": PREC_BF16,
              "f16x3": PREC_F16X3}  # f16x3: forward only (its backward runs bf16x6)


def jet_prec(p):
    """INSR_JET_PREC(p): the per-call precision bits OR-ed into a jet `mode`."""
    return (int(p) + 1) << MODE_PREC_SHIFT


MODE_BPREC_SHIFT = 12


def jet_bprec(p):
    """INSR_JET_BPREC(p): a backward-only precision override OR-ed into a jet `mode`."""
    return (int(p) + 1) << MODE_BPREC_SHIFT


# Per-call knobs (include/insr_siren.h INSR_JET_POLICY / INSR_JET_BWD_F16 / INSR_JET_TILES /
# INSR_MODE_WIDE128): bits of the `mode` argument.  The library keeps no mutable configuration.
ERANGE = -5  # INSR_ERANGE
MODE_WIDE128 = 1 << 9
MODE_POLICY_SHIFT, MODE_F16_SHIFT, MODE_TILES_SHIFT = 16, 19, 23
BWD_F16_DW, BWD_F16_PROP, BWD_F16_FUSED = 1, 2, 4
_TCODE = {0: 0, 1: 1, 2: 2, 4: 3}
_MINB = {256: 0, 512: 1, 128: 2, 1024: 3}
_PREC_BITS = (0xF << MODE_PREC_SHIFT) | (0xF << MODE_BPREC_SHIFT)
_FIELDS = {"policy": 7 << MODE_POLICY_SHIFT, "bwd_f16": 0xF << MODE_F16_SHIFT, "tiles": 0x3F << MODE_TILES_SHIFT,
           "wide128": MODE_WIDE128, "prec": _PREC_BITS}


def jet_policy(p):
    """INSR_JET_POLICY(p): backward path 0 auto, 1 fused, 2 two-kernel, 3 resident dW (bf16x6), 4 recompute,
    5 resident dW with f16x3 products (the recompute kernel's reverse sweep on the saved streams)."""
    return (int(p) + 1) << MODE_POLICY_SHIFT


def jet_bwd_f16(mask):
    """INSR_JET_BWD_F16(mask): the x6 backward's products on the fp16 matrix cores (BWD_F16_* bits)."""
    return (int(mask) + 1) << MODE_F16_SHIFT


def jet_tiles(fwd=0, bwd=0, min_blocks=256):
    """INSR_JET_TILES: forced tiles per block (0 auto, 1, 2, 4) and the auto choice's minimum block count."""
    return (_TCODE[int(fwd)] | (_TCODE[int(bwd)] << 2) | (_MINB[int(min_blocks)] << 4)) << MODE_TILES_SHIFT


def knob_bits(policy=None, bwd_f16=None, tiles=None, wide128=None, prec=None):
    """Mode bits of the given knobs (None: the field stays at the library default).
    tiles = (fwd, bwd[, min_blocks]); prec = (fwd, bwd) INSR_PREC_* codes."""
    b = 0
    if policy is not None:
        b |= jet_policy(policy)
    if bwd_f16 is not None:
        b |= jet_bwd_f16(bwd_f16)
    if tiles is not None:
        b |= jet_tiles(*tiles)
    if wide128:
        b |= MODE_WIDE128
    if prec is not None:
        b |= jet_prec(prec[0]) | jet_bprec(prec[1])
    return b


# A knob scope of the calling thread: the bits base.MLP.call_mode adds to the jets it launches
# (forward time: the backward of a jet reuses its forward's mode, so the two always agree).
# A network's own precision (MLP(precision=...)) wins over a scope's `prec`.
_scope = threading.local()


def scope_bits():
    return getattr(_scope, "bits", 0)


def _merged(old, kw):
    clear = 0
    for k, v in kw.items():
        if v is not None:
            clear |= _FIELDS[k]
    return (old & ~clear) | knob_bits(**kw)


def set_default_knobs(**kw):
    """The calling thread's knob scope for the rest of its life (drivers: bench.py, tools/)."""
    _scope.bits = _merged(scope_bits(), kw)
    return _scope.bits


def bwd_f16_mask(bits=None):
    """The INSR_BWD_F16_* mask a call with these mode bits (default: the scope's) runs with."""
    f = ((scope_bits() if bits is None else bits) >> MODE_F16_SHIFT) & 0xF
    return f - 1 if f else BWD_F16_DW | BWD_F16_PROP | BWD_F16_FUSED


@contextlib.contextmanager
def knobs(**kw):
    """with knobs(policy=4, bwd_f16=0, tiles=(1, 4, 512), wide128=True, prec=(1, 1)): ... -- A/B
    studies and tests; fields not named keep the enclosing scope's value."""
    old = scope_bits()
    _scope.bits = _merged(old, kw)
    try:
        yield _scope.bits
    finally:
        _scope.bits = old
LOSS_COMBO, LOSS_BANDS = 0, 1
OPT_LR, OPT_STEP, OPT_BEST, OPT_BAD, OPT_STEPSIZE, OPT_BC2SQRT, OPT_FACTOR, OPT_MINLR = range(8)
OPT_TICKET = 8  # the fused Adam + plateau launch's last-block ticket (0 between launches)
OPT_TICKET_SHARDS = 9  # [9, 17): its first-level shards (0 between launches)
OPT_NFLOATS = 17
ADAM_MAX_TENSORS = 8

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_long
_F = ctypes.c_float

# name -> (restype, argtypes); mirrors include/insr_siren.h one to one
SIGNATURES = {
    "insr_version": (_I, []),
    "insr_build_id": (ctypes.c_char_p, []),
    "insr_siren_param_count": (_L, [_I, _I, _I, _I]),
    "insr_siren_supported": (_I, [_I, _I, _I, _I, _I]),
    "insr_jet_act_bytes": (_L, [_L, _I, _I, _I, _I]),
    "insr_jet_partial_bytes": (_L, [_L, _I, _I, _I, _I, _I]),
    "insr_siren_jet_fwd": (_I, [_P, _L, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P]),
    "insr_siren_jet_fwd_multi": (_I, [_P, _I, _I, _I, _I, _I, _I, _P]),
    "insr_siren_jet_bwd": (_I, [_P, _L, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P]),
    "insr_jet_partial_blocks": (_I, [_L, _I, _I, _I]),
    "insr_siren_jet_bwd_grad": (_I, [_P, _L, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _I, _P]),
    "insr_jet_bwd_work_bytes": (_L, [_L, _I, _I, _I, _I, _I]),
    "insr_siren_jet_bwd_grad_multi": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _P, _P, _I, _P]),
    "insr_jet_bwd_multi_work_bytes": (_L, [_P, _I, _I, _I, _I, _I, _I]),
    "insr_siren_jet_bwd_multi_rows": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _P, _P]),
    "insr_siren_jet_bwd_multi_sweep": (_I, [_P, _I, _I, _I, _I, _I, _I, _P, _P, _P]),
    "insr_jet_bwd_is_wide": (_I, [_L, _I, _I, _I]),
    "insr_jet_bwd_path": (_I, [_L, _I, _I, _I, _I, _I]),
    "insr_jet_bwd_kernel": (_I, [_L, _I, _I, _I, _I, _I]),
    "insr_comm_available": (_I, []),
    "insr_comm_id_bytes": (_L, []),
    "insr_comm_unique_id": (_I, [_P]),
    "insr_comm_init": (_I, [_P, _I, _I, _P]),
    "insr_comm_allreduce_sum": (_I, [_P, _P, _L, _P]),
    "insr_comm_destroy": (_I, [_P]),
    "insr_jet_split_tiles": (_I, [_L, _I, _I, _I, _I]),
    "insr_sq_loss_work_floats": (_L, []),
    "insr_svd_energy_work_floats": (_L, []),
    "insr_svd_energy_fwd": (_I, [_P, _L, _I, _F, _F, _P, _P, _P]),
    "insr_svd_energy_bwd": (_I, [_P, _L, _I, _F, _F, _P, _P, _P]),
    "insr_elastic_work_floats": (_L, []),
    "insr_elastic_energy": (_I, [_P, _P, _P]),
    "insr_sq_loss_fwd": (_I, [_I, _P, _P, _P, _P, _L, _I, _F, _F, _F, _F, _F, _P, _P, _P]),
    "insr_sq_loss_group": (_I, [_P, _I, _P, _P]),
    "insr_axpy_clamp": (_I, [_P, _P, _F, _F, _F, _P, _L, _P]),
    "insr_siren_wsplit_offset": (_L, [_I, _I, _I, _I]),
    "insr_siren_wsplit_floats": (_L, [_I, _I]),
    "insr_siren_wsplit": (_I, [_P, _I, _I, _I, _I, _P]),
    "insr_siren_wsplit_status": (_I, [_P, _I, _I, _I, _I, _P]),
    "insr_siren_jet_fwd_mixed": (_I, [_P, _P, _P, _I, _I, _I, _I, _I, _I, _P]),
    "insr_adam_step_nets": (_I, [_I, _P, _P, _P, _P, _P, _P, _P, _F, _F, _F, _I, _P]),
    "insr_adam_plateau_step_nets": (_I, [_I, _P, _P, _P, _P, _P, _P, _P, _F, _F, _F, _P, _I, _P]),
    "insr_adam_step_partials": (_I, [_P, _I, _L, _P, _I, _P, _P, _P, _L, _P, _P, _F, _F, _F, _P, _I, _P]),
    "insr_siren_jet_bwd_grad_adam": (_I, [_P, _L, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _P, _I, _I, _P, _P, _P,
                                          _F, _F, _F, _P, _I, _P]),
    "insr_jet_wide_launch_threads": (_I, [_L, _I, _I, _I, _I, _I, _P]),
    "insr_sq_loss_bwd": (_I, [_I, _P, _P, _P, _P, _L, _I, _F, _F, _F, _F, _F, _P, _P, _P, _P, _P, _P]),
    "insr_reduce_partials": (_I, [_P, _I, _L, _P, _I, _P]),
    "insr_reduce_partials_strided": (_I, [_P, _I, _L, _L, _P, _I, _P]),
    "insr_jet_partial_stride": (_L, [_I, _I, _I, _I]),
    "insr_adam_prepare": (_I, [_P, _F, _F, _P]),
    "insr_plateau_step": (_I, [_P, _P, _I, _I, _P]),
    "insr_adam_step_multi": (_I, [_I, _P, _P, _P, _P, _P, _P, _F, _F, _F, _I, _P]),
    "insr_sampler_state_bytes": (_L, []),
    "insr_sample_boxes": (_I, [_P, _I, _I, ctypes.c_ulonglong, _P, _P]),
    "insr_sample_boxes_rep": (_I, [_P, _I, _I, _I, _P, ctypes.c_ulonglong, _P, _P]),
    "insr_advect1d_rows": (_L, [_L]),
    "insr_advect1d_iteration": (_I, [_P, _P, _I, _I, _L, _L, _P, _P, _F, _F, _F, _F, ctypes.c_ulonglong, _P, _P,
                                     _P, _L, _P, _P, _P]),
    "insr_adam_step": (_I, [_P, _P, _P, _P, _L, _P, _F, _F, _F, _P]),
    "insr_jet_bwd_seed_rows": (_I, [_L, _I, _I, _I, _I, _I]),
    "insr_siren_jet_bwd_seeded": (_I, [_P, _L, _I, _I, _I, _I, _I, _P, _P, _P, _P, _P, _P, _I, _P, _P, _P]),
    "insr_reduce_partials_fin": (_I, [_P, _I, _L, _L, _P, _I, _P, _P]),
    "insr_adam_step_partials_fin": (_I, [_P, _I, _L, _P, _I, _P, _P, _P, _L, _P, _P, _F, _F, _F, _P, _I, _P, _P]),
    "insr_siren_jet_bwd_grad_adam_fin": (_I, [_P, _L, _I, _I, _I, _I, _I, _P, _P, _P, _I, _P, _P, _P, _F, _F, _F, _P,
                                              _I, _P, _P]),
}


MAX_FWD_JOBS = 6  # INSR_MAX_FWD_JOBS


class JetJob(ctypes.Structure):
    """struct InsrJetJob (include/insr_siren.h): one forward jet of insr_siren_jet_fwd_multi."""
    _fields_ = [("x", _P), ("params", _P), ("y", _P), ("dy", _P), ("lap", _P), ("act", _P), ("n", _L), ("d_out", _I)]


MAX_BWD_JOBS = 8  # INSR_MAX_BWD_JOBS


class BwdJob(ctypes.Structure):
    """struct InsrBwdJob (include/insr_siren.h): one backward job of insr_siren_jet_bwd_grad_multi."""
    _fields_ = [("x", _P), ("act", _P), ("gy", _P), ("gdy", _P), ("glap", _P), ("n", _L)]


LOSS_GROUP_MAX = 4  # INSR_LOSS_GROUP_MAX


class Loss(ctypes.Structure):
    """struct InsrLoss (include/insr_siren.h): one loss of insr_sq_loss_group."""
    _fields_ = [("kind", _I), ("m", _I), ("n", _L), ("a", _P), ("b", _P), ("c", _P), ("d", _P),
                ("sb", _L), ("sc", _L), ("sd", _L),
                ("alpha", _F), ("beta", _F), ("gamma", _F), ("delta", _F), ("scale", _F), ("out", _P),
                ("ga", _P), ("ga_lo", _L), ("ga_hi", _L), ("a_off", _L), ("gb", _P), ("gc", _P), ("gd", _P),
                ("gb_len", _L), ("gc_len", _L), ("gd_len", _L)]


SEED_MAX = 4  # INSR_SEED_MAX
SEED_VALUE, SEED_GRAD, SEED_LAP = 0, 1, 2  # INSR_SEED_VALUE / _GRAD / _LAP


class Seed(ctypes.Structure):
    """struct InsrSeed (include/insr_siren.h): one loss term a reverse jet evaluates as its adjoint."""
    _fields_ = [("kind", _I), ("m", _I), ("stream", _I), ("loss", _I), ("n", _L), ("a_off", _L),
                ("a", _P), ("b", _P), ("c", _P), ("d", _P), ("sb", _L), ("sc", _L), ("sd", _L),
                ("alpha", _F), ("beta", _F), ("gamma", _F), ("delta", _F), ("scale", _F)]


class LossFin(ctypes.Structure):
    """struct InsrLossFin (include/insr_siren.h): the loss values a sums launch finishes."""
    _fields_ = [("part", _P), ("rows", _I), ("nloss", _I), ("scale", _F * SEED_MAX), ("out", _P * SEED_MAX)]


MAX_BOXES = 8  # INSR_MAX_BOXES


class Box(ctypes.Structure):
    """struct InsrBox (include/insr_siren.h): one box of insr_sample_boxes."""
    _fields_ = [("out", _P), ("n", _L), ("lo", _F * 3), ("hi", _F * 3)]


EL_TERMS = 8  # INSR_EL_TERMS; term ids INSR_EL_ARAP ... INSR_EL_SPHERE
EL_IDS = {"arap": 0, "volume": 1, "kinematics": 2, "external": 3, "constraint": 4, "constraint_right": 5,
          "collision": 6, "collision_sphere": 7}


class Elastic(ctypes.Structure):
    """struct InsrElastic (include/insr_siren.h): one elasticity energy of insr_elastic_energy."""
    _fields_ = [("d", _I), ("n_order", _I), ("n", _L), ("rows", _L), ("f", _P), ("J", _P), ("x", _P),
                ("f_prev", _P), ("f_pp", _P), ("dt", _F), ("ratio", _F * EL_TERMS), ("ext", _F * 3),
                ("target", _F * 3), ("plane_height", _F), ("center", _F * 3), ("radius", _F),
                ("row_l", _L), ("n_l", _L), ("row_r", _L), ("n_r", _L), ("order", _I * EL_TERMS),
                ("out", _P), ("terms", _P), ("gf", _P), ("gJ", _P)]


class NativeUnavailable(RuntimeError):
    pass


class NativeError(RuntimeError):
    pass


_lib = None
_load_error = None

CSRC = os.path.join(os.path.dirname(_HERE), "csrc")
HEADER = os.path.join(os.path.dirname(os.path.dirname(_HERE)), "include", "insr_siren.h")


def source_hash():
    """What insr_build_id() must return for a library built from the checked-out sources
    (the recipe of csrc/Makefile's SRC_HASH); None when the sources are not present."""
    import glob
    import hashlib
    names = sorted(os.path.basename(p) for p in glob.glob(os.path.join(CSRC, "*.hip")) +
                   glob.glob(os.path.join(CSRC, "*.hpp")))
    if not names or not os.path.exists(HEADER):
        return None
    h = hashlib.sha256()
    for p in [os.path.join(CSRC, n) for n in names] + [HEADER]:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def load(path=None, check_build=True):
    """Load (once) and return the CDLL with typed signatures.  check_build=False only for
    study tools that load an explicit alternative build (tools/kbench.py --lib)."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        _load_error = f"{p} not found: run `python -c 'import __graft_entry__ as g; g.build()'`"
        raise NativeUnavailable(_load_error)
    lib = ctypes.CDLL(p)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:
            if check_build:
                raise NativeUnavailable(f"{p} does not export {name}: rebuild")
            continue  # an older study build (tools/kbench.py --lib): its missing entries stay unused
        fn.restype = res
        fn.argtypes = args
    want, have = source_hash(), lib.insr_build_id().decode()
    if check_build and want is not None and want != have:
        _load_error = (f"{p} was built from other sources (build id {have}, checked-out sources {want}): "
                       "rebuild with `python -c 'import __graft_entry__ as g; g.build()'`")
        raise NativeUnavailable(_load_error)
    _lib = lib
    return lib


def lib():
    return _lib if _lib is not None else load()


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_of(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def check(rc, what):
    if rc != 0:
        raise NativeError(f"{what} failed with code {rc}")
