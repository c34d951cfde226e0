"""ddpca-admm_amd: MI355X-native hot path of DDPCA-ADMM (per-subdomain solve loop of the ADMM).

Python mirror of the reference's class surface for this path -- ``MULTIGRID`` (MULTIGRID.h:10-95),
``MGPIS`` (MGPIS.h:8-38) and ``MCONTACT`` (MCONTACT.h:9-95) -- over the C ABI of
``libddpca_amd.so`` (include/ddpca_amd.h).  All compute runs in the HIP library; this module only
marshals arrays.  There is no CPU fallback: if the library is missing or no gfx950 GPU is visible,
the device entry points raise.

The package directory name contains a hyphen, so import it with
``importlib.import_module("ddpca-admm_amd")`` (see ``__graft_entry__.py``).
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path
from typing import Optional, Sequence

import numpy as np

_HERE = Path(__file__).resolve().parent
# DDPCA_AMD_LIB: an in-tree experiment build (build.py with DDPCA_BUILD_OUT) for kernel A/B runs
LIBPATH = Path(os.environ.get("DDPCA_AMD_LIB", _HERE / "libddpca_amd.so"))

_lib: Optional[C.CDLL] = None


class DdpcaError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[ddpca error {code}] {msg}")
        self.code = code


def lib() -> C.CDLL:
    """Load libddpca_amd.so (built in-tree by build.py); raise loudly if it is missing."""
    global _lib
    if _lib is None:
        if not LIBPATH.exists():
            raise ImportError(f"{LIBPATH} is missing: run `python ddpca-admm_amd/build.py` (hipcc, gfx950)")
        _lib = C.CDLL(str(LIBPATH), mode=C.RTLD_GLOBAL)
        _declare(_lib)
    return _lib


class MgpisOptions(C.Structure):
    _fields_ = [("smoother", C.c_int), ("nu", C.c_int), ("omega", C.c_double), ("iters_per_graph", C.c_int),
                ("warm_start", C.c_int), ("precond_fp32", C.c_int), ("table_mode", C.c_int),
                ("coarse_level", C.c_int)]


# The option set bench.py measures the headline on (its defaults; tests/test_headline_gpu.py pins
# this exact set against the oracle): multicolour block Gauss-Seidel on the fine level (one
# forward sweep before, one backward after the coarse correction), 3x3 block-Jacobi with two
# sweeps (damping 1.7 / lambda_max) on the levels below, V-cycle levels stored fp32 with the three
# finest as block-scaled int8 (nine int8 and a scale per 3x3 block), streamed operator rows,
# automatic exact-solve level, 4 PCG iterations per hipGraph replay, x0 = 0.  (18.0 instead of
# block-Jacobi V(1,1)'s 23.6 PCG iterations per solve, +8-10 % ADMM it/s at 8 subdomains per GPU,
# +5 % at 4, equal at 2: profiles/r03j; round 4: +10 % at 4, +4 % at 2,
# profiles/r04l/ab_small_batch.txt.  The int8 copies instead of block-exponent fp16: 18.6 instead
# of 18.0 PCG iterations, +6 % ADMM it/s, the one-subdomain rank -7.5 %, profiles/r05r.  Round 6:
# precond_fp32 = 4 -- the same int8 copies, and the fine colour sweeps gather an fp32 stride-4 copy of
# the iterate and restrict an fp32 copy of their residual: the same 18.6 PCG iterations, 18.93 ->
# 19.74 ADMM it/s alternating in one call, profiles/r06d; the block-Jacobi levels below on fp32
# iterate copies too: 19.73 -> 20.05 ADMM it/s, the N = 8 rank 9.52 -> 9.00 ms, profiles/r06n.
# Colour SSOR on the fine level (smoother 4, the reference's smoothing order) took 17.6 iterations
# at 59 instead of 50.6 ms, profiles/r06e.)
HEADLINE_OPTIONS = dict(smoother=3, nu=2, omega=-1.7, iters_per_graph=4, warm_start=0, precond_fp32=4,
                        table_mode=0, coarse_level=-1)
# ... for a rank that owns at most 4 subdomains (the 2-, 4- and 8-GPU runs of the same chain): a
# colour launch then holds <= 1,600 chunks and the 17 fine-level launches per V-cycle are
# latency-bound, so block Jacobi with two sweeps per level, pinned by the same tests.  Round 5, on
# the int8 copies (profiles/r05y, one rank of each layout under the loopback transport, ms per ADMM
# iteration): 1 subdomain 9.50 (17 PCG iterations) against 9.93 with one sweep (24), 9.80 with three
# (14) and 11.33 for the multicolour set (19); 2 subdomains 15.34 vs multicolour 16.47; 4 subdomains
# 27.95 vs 28.72; at 8 the multicolour set leads, 18.98 vs 18.28 ADMM it/s.  (Before the int8
# copies the one-sweep set was the small one: profiles/r03j, r04l.)
HEADLINE_OPTIONS_SMALL = dict(HEADLINE_OPTIONS, smoother=1, nu=2)


def headline_options(n_owned: int) -> dict:
    """The measured-best headline option set for a rank owning n_owned subdomains."""
    return dict(HEADLINE_OPTIONS if n_owned > 4 else HEADLINE_OPTIONS_SMALL)
# and the ADMM setting it runs: interface-eliminated coarse space (muscSett = 2) on level 1 of
# every subdomain (DEHW.h:2222, 2239)
HEADLINE_MUSC = dict(muscSett=2, doleMcsc=1)
# and the workload: the synthetic DEHW chain of bench.py (4 worm/wheel groups = 8 subdomains,
# 3x2x2 coarse hexes refined gl = 5 times, Coulomb mu = 0.2) at SURVEY §8 d2 M3's interface
# density -- contact faces integrated over 2^2 x 2^2 polygons, glued faces over 2^1 x 2^1
# (0.80 integration points per DOF at gl = 5).  bench.py's defaults and the headline parity tests
# (tests/test_headline_gpu.py, at gl = 3 for the oracle trajectory) both take it from here.
HEADLINE_WORKLOAD = dict(groups=4, nx=3, ny=2, nz=2, gl=5, fric=0.2, ip_contact=2, ip_glued=1, band=0, rot=0)
# DEHW's general-mesh features on the same chain (bench.py --mesh general): the contact band refined
# once more (a general tree: hanging level past the MGPIS hierarchy, explicit transfer lists) and
# rotated support nodes (prolongation blocks off w I); the same coarse space as the headline
# (HEADLINE_MUSC: MULTISCALE_1 on the general tree, multiscale.cpp)
GENERAL_FEATURES = dict(band=1, rot=1)


def headline_problem(gl: int | None = None, **override) -> "Problem":
    """The bench's DEHW-synthetic Problem (HEADLINE_WORKLOAD), optionally at another refinement
    depth or with other workload parameters."""
    w = dict(HEADLINE_WORKLOAD, **override)
    if gl is not None:
        w["gl"] = gl
    return Problem("dehw", w["groups"], w["nx"], w["ny"], w["nz"], w["gl"], w["fric"], w["ip_contact"],
                   w["ip_glued"], w["band"], w["rot"], w.get("uneven", 0))

_P = C.c_void_p
_I64P = C.POINTER(C.c_int64)
_DP = C.POINTER(C.c_double)


class _CsrArg(C.Structure):  # ddpca_csr_t
    _fields_ = [("nrow", C.c_int64), ("ncol", C.c_int64), ("ptr", C.c_void_p), ("col", C.c_void_p),
                ("val", C.c_void_p)]


def _declare(L: C.CDLL) -> None:
    L.ddpca_last_error.restype = C.c_char_p
    L.ddpca_gpu_available.restype = C.c_int
    L.mgpis_default_options.argtypes = [C.POINTER(MgpisOptions)]
    L.mgpis_default_options.restype = None
    L.ddpca_problem_create.argtypes = [C.c_char_p, _DP, C.c_int, C.POINTER(_P)]
    L.ddpca_problem_set_ips.argtypes = [_P, C.c_int64, C.c_int64, _P, _P, _P, _P, _P, C.c_double, C.c_double,
                                        C.c_double]
    L.ddpca_problem_establish.argtypes = [_P]
    L.ddpca_problem_set_coarse.argtypes = [_P, C.c_int64, _P]
    L.ddpca_contact_search.argtypes = [_P, C.c_int64, _P, C.c_int64, C.c_int64, _P, _P, C.c_int64, _P, _P, _P,
                                       C.c_double, C.POINTER(_P)]
    L.ddpca_refine_select.argtypes = [_P, C.c_int64, _P, C.c_int64, C.c_int64, _P, _P, C.c_int64, _P, _P, _P,
                                      C.c_double, C.c_int64, _P, C.c_int64, _P, _P, _P]
    L.ddpca_ips_count.argtypes = [_P]
    L.ddpca_ips_count.restype = C.c_int64
    L.ddpca_ips_get.argtypes = [_P, _P, _P, _P, _P, _P]
    L.ddpca_ips_destroy.argtypes = [_P]
    L.ddpca_problem_establish_owned.argtypes = [_P, _P, C.c_int]
    L.ddpca_lagrange_create.argtypes = [C.c_int64, C.c_int64, C.POINTER(_P)]
    L.ddpca_lagrange_set_subdomain.argtypes = [_P, C.c_int64, C.c_int, _P, _P, _P, C.POINTER(_CsrArg),
                                               C.POINTER(_CsrArg), _P, C.c_int64, C.POINTER(_CsrArg), _P]
    L.ddpca_lagrange_set_interface.argtypes = [_P, C.c_int64, C.c_int64, C.c_int64, C.c_double, C.c_int64, _P, _P,
                                               _P, _P, _P]
    L.ddpca_lagrange_solve.argtypes = [_P, C.c_int, C.c_int, C.POINTER(MgpisOptions), C.c_int64]
    L.ddpca_lagrange_solve.restype = C.c_int64
    L.ddpca_lagrange_get.argtypes = [_P, C.c_char_p, C.c_int64, _P, C.c_int64]
    L.ddpca_lagrange_get.restype = C.c_int64
    L.ddpca_lagrange_destroy.argtypes = [_P]
    L.ddpca_problem_view.argtypes = [_P, C.c_char_p, C.c_int64, C.c_int64, C.POINTER(_P), _I64P,
                                     C.POINTER(C.c_int)]
    L.ddpca_problem_destroy.argtypes = [_P]
    L.ddpca_problem_mgpis.argtypes = [_P, C.c_int64, C.c_int, C.POINTER(MgpisOptions), C.POINTER(_P)]
    L.ddpca_problem_empty.argtypes = [C.c_int64, C.c_int64, C.POINTER(_P)]
    L.ddpca_problem_set_contact.argtypes = [_P, C.c_int64, C.c_int64, C.c_int64]
    L.ddpca_problem_set_subdomain_tree.argtypes = [_P, C.c_int64, _P]
    L.ddpca_problem_set_subdomain.argtypes = [_P, C.c_int64, C.c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]
    L.ddpca_problem_set_subdomain_prol.argtypes = [_P, C.c_int64, C.c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                                   _P]
    L.ddpca_problem_set_hanging.argtypes = [_P, C.c_int64, C.c_int64, C.POINTER(_CsrArg)]
    L.ddpca_problem_set_interface.argtypes = [_P, C.c_int64, C.c_int64, C.c_int64, C.c_double, C.c_int64, C.c_int64,
                                              C.c_int64, _P, _P, C.POINTER(_CsrArg)]
    L.ddpca_problem_finalize.argtypes = [_P]
    L.ddpca_problem_set_coarse_operators.argtypes = [_P, C.c_int64, _P, _P, C.POINTER(_CsrArg), _P,
                                                     C.POINTER(_CsrArg), C.POINTER(_CsrArg), C.POINTER(_CsrArg)]
    L.ddpca_problem_set_coarse_nodes.argtypes = [_P, C.c_int64, C.c_int64, _P]
    L.ddpca_problem_set_coarse_latin.argtypes = [_P, _P, _P, C.POINTER(_CsrArg), C.POINTER(_CsrArg),
                                                 C.POINTER(_CsrArg), C.POINTER(_CsrArg), C.POINTER(_CsrArg)]
    L.mgpis_gpu_create.argtypes = [C.c_int, C.c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                   C.POINTER(MgpisOptions), C.POINTER(_P)]
    L.mgpis_gpu_create_prol.argtypes = [C.c_int, C.c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                        C.POINTER(MgpisOptions), C.POINTER(_P)]
    L.mgpis_gpu_create_bsr3.argtypes = [C.c_int, C.c_int, _P, _P, _P, _P, _P, _P, _P, _P,
                                        C.POINTER(MgpisOptions), C.POINTER(_P)]
    L.mgpis_gpu_solve.argtypes = [_P, _P, _P, C.c_int, C.c_double, C.c_int64, _I64P, _DP]
    L.mgpis_gpu_mult_solve.argtypes = [_P, _P, _P, C.c_int64, _I64P, _DP]
    L.mgpis_gpu_bicgstab.argtypes = [_P, _P, _P, C.c_int, C.c_double, C.c_int64, _I64P, _DP,
                                     C.POINTER(C.c_int)]
    L.mgpis_gpu_gmres.argtypes = [_P, _P, _P, C.c_int, C.c_double, C.c_int64, C.c_int64, _I64P, _DP]
    L.mgpis_gpu_spmv.argtypes = [_P, C.c_int, _P, _P]
    L.mgpis_gpu_spmv_copy.argtypes = [_P, C.c_int, C.c_int, _P, _P]
    L.ddpca_write_resuDisp.argtypes = [C.c_char_p, _P, C.c_int64, C.c_int64, _P, _P]
    L.ddpca_write_resuCont.argtypes = [C.c_char_p, C.c_double, C.c_int64, _P, _P, _P]
    L.ddpca_write_resuMoni.argtypes = [C.c_char_p, _P, C.c_int64, C.c_int64]
    L.mgpis_gpu_vcycle.argtypes = [_P, _P, _P]
    L.mgpis_gpu_info.argtypes = [_P, _I64P]
    L.mgpis_gpu_bench_spmv.argtypes = [_P, C.c_int, C.c_int, _DP, _DP]
    L.mgpis_gpu_destroy.argtypes = [_P]
    if hasattr(L, "mcontact_gpu_create"):
        L.mcontact_gpu_create.argtypes = [_P, C.c_int, C.c_int, C.c_int, _P, C.POINTER(MgpisOptions),
                                          C.POINTER(_P)]
        L.mcontact_gpu_comm_init.argtypes = [_P, _P]
        L.mcontact_gpu_comm_local.argtypes = [_P, C.c_int]
        L.mcontact_gpu_comm_loopback.argtypes = [_P, _P]
        L.mcontact_gpu_unique_id.argtypes = [_P]
        L.mcontact_gpu_iterate.argtypes = [_P, C.c_int64, C.c_int]
        L.mcontact_gpu_iterate.restype = C.c_int64
        L.mcontact_gpu_monitor.argtypes = [_P, _DP, C.c_int64]
        L.mcontact_gpu_monitor.restype = C.c_int64
        L.mcontact_gpu_get.argtypes = [_P, C.c_char_p, C.c_int64, _P, C.c_int64]
        L.mcontact_gpu_get.restype = C.c_int64
        L.mcontact_gpu_timing.argtypes = [_P, _DP]
        L.mcontact_gpu_bytes.argtypes = [_P, _DP, C.c_int64]
        L.mcontact_gpu_bytes.restype = C.c_int64
        L.mcontact_gpu_destroy.argtypes = [_P]
        L.mcontact_gpu_comm_check.argtypes = [_P, C.c_int64]
        L.ddpca_mass_solve.argtypes = [C.c_int, C.c_int64, C.POINTER(_CsrArg), _P, _P, C.c_double, C.c_int64, C.c_int,
                                       _P]


def _check(rc: int) -> int:
    if rc < 0:
        raise DdpcaError(rc, lib().ddpca_last_error().decode())
    return rc


def gpu_available() -> bool:
    return bool(lib().ddpca_gpu_available())


_probe_lib = None


def probe_lib() -> C.CDLL:
    """libddpca_probe.so (include/ddpca_probe.h): the measurement probes beside the product."""
    global _probe_lib
    if _probe_lib is None:
        lib()  # the probe library resolves its error plumbing from the product library
        path = Path(LIBPATH).with_name("libddpca_probe.so")
        if not path.exists():
            raise ImportError(f"{path} is missing: run ddpca-admm_amd/build.py")
        L = C.CDLL(str(path))
        L.ddpca_stream_ceiling.argtypes = [C.c_int, C.c_int64, C.c_int, _DP]
        L.ddpca_probe_grid_barrier.argtypes = [C.c_int, C.c_int64, C.c_int, C.c_int, C.c_int, _DP]
        _probe_lib = L
    return _probe_lib


def stream_ceiling(device: int = 0, nbytes: int = 2 << 30, reps: int = 10) -> dict:
    """This box's STREAM copy / read bandwidth (ddpca_stream_ceiling), in GB/s."""
    out = (C.c_double * 4)()
    _check(probe_lib().ddpca_stream_ceiling(device, int(nbytes), int(reps), out))
    return dict(copy_gbs=out[0], read_gbs=out[1], copy_ms=out[2], read_ms=out[3], bytes_per_buffer=int(nbytes))


def probe_grid_barrier(n: int, phases: int = 64, blocks: int = 256, pin: bool = False, device: int = 0) -> dict:
    """Graph kernel boundary vs persistent grid barrier per dependent pass over n doubles
    (ddpca_probe_grid_barrier; measurement only); pin: the persistent workgroups on one XCD."""
    out = (C.c_double * 4)()
    _check(probe_lib().ddpca_probe_grid_barrier(device, int(n), int(phases), int(blocks), int(bool(pin)), out))
    return dict(graph_us=out[0], persistent_us=out[1], max_diff=out[2], timed_out=int(out[3]))


def default_options(**kw) -> MgpisOptions:
    o = MgpisOptions()
    lib().mgpis_default_options(C.byref(o))
    for k, v in kw.items():
        setattr(o, k, v)
    return o


def _ptr(a: np.ndarray) -> C.c_void_p:
    return C.c_void_p(a.ctypes.data)


_DTYPES = {0: np.float64, 1: np.int64, 2: np.int32, 3: np.uint8}


# ============================================================================ host problem
class Problem:
    """Host problem (MULTIGRID meshes + MCONTACT interfaces); setup only.

    kind/params: ``beam`` (d0, d1, d2, globLeve, D0, D1, D2), ``twoblock`` (fric, globLeve),
    ``dehw`` (ngroups, nx, ny, nz, globLeve, fric).
    """

    def __init__(self, kind: str, *params: float):
        p = np.asarray(params, dtype=np.float64)
        h = C.c_void_p()
        _check(lib().ddpca_problem_create(kind.encode(), p.ctypes.data_as(_DP), len(p), C.byref(h)))
        self._h = h
        self.kind = kind

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.ddpca_problem_destroy(h)
            self._h = None

    @property
    def handle(self) -> C.c_void_p:
        return self._h

    def array(self, name: str, index: int = 0, level: int = 0) -> np.ndarray:
        data = C.c_void_p()
        count = C.c_int64()
        dt = C.c_int()
        _check(lib().ddpca_problem_view(self._h, name.encode(), index, level, C.byref(data), C.byref(count),
                                        C.byref(dt)))
        dtype = np.dtype(_DTYPES[dt.value])
        if count.value == 0:
            return np.zeros(0, dtype)
        buf = (C.c_char * (count.value * dtype.itemsize)).from_address(data.value)
        return np.frombuffer(buf, dtype=dtype).copy()

    def csr(self, base: str, index: int = 0, level: int = 0):
        import scipy.sparse as sp
        shape = tuple(self.array(f"{base}:shape", index, level))
        return sp.csr_matrix((self.array(f"{base}:val", index, level), self.array(f"{base}:col", index, level),
                              self.array(f"{base}:ptr", index, level)), shape=shape)

    @property
    def nsub(self) -> int:
        return int(self.array("sizes")[0])

    @property
    def nint(self) -> int:
        return int(self.array("sizes")[1])

    def set_ips(self, ts: int, node, shap, basis, gap, w, fric: float, penN: float, penF: float) -> None:
        """Replace interface ts's integration points (CSEARCH::intePoin data contract)."""
        node = np.ascontiguousarray(node, dtype=np.int64)
        shap = np.ascontiguousarray(shap, dtype=np.float64)
        basis = np.ascontiguousarray(basis, dtype=np.float64)
        gap = np.ascontiguousarray(gap, dtype=np.float64)
        w = np.ascontiguousarray(w, dtype=np.float64)
        _check(lib().ddpca_problem_set_ips(self._h, ts, len(gap), _ptr(node), _ptr(shap), _ptr(basis), _ptr(gap),
                                           _ptr(w), fric, penN, penF))

    def set_coarse(self, muscSett: int, doleMcsc: Optional[Sequence[int]] = None) -> "Problem":
        """MCONTACT::muscSett / doleMcsc (MCONTACT.h:22-23) before ESTABLISH; 2 = the
        interface-eliminated coarse space (MULTISCALE_1)."""
        d = None if doleMcsc is None else np.ascontiguousarray(doleMcsc, dtype=np.int64)
        _check(lib().ddpca_problem_set_coarse(self._h, int(muscSett), None if d is None else _ptr(d)))
        self._keep_dole = d
        return self

    def ESTABLISH(self, owner: Optional[Sequence[int]] = None, rank: int = 0) -> "Problem":
        """MCONTACT::ESTABLISH; with owner/rank only this rank's subdomains are built."""
        if owner is None:
            _check(lib().ddpca_problem_establish(self._h))
        else:
            own = np.ascontiguousarray(owner, dtype=np.int32)
            _check(lib().ddpca_problem_establish_owned(self._h, _ptr(own), rank))
        return self

    def grid(self, tv: int = 0) -> "MULTIGRID":
        return MULTIGRID(self, tv)

    # ---- operator-level builder (ddpca_problem_empty / set_subdomain / set_interface / finalize)
    IFACE_OPS = ("inpoLagr", "pemaInpo_r", "systTran", "systTran_pena", "inteMass", "inteMass_pena", "inteInpo")

    @classmethod
    def from_operators(cls, subdomains: Sequence[dict], interfaces: Sequence[dict],
                       coarse: Optional[dict] = None) -> "Problem":
        """Established problem from operators in the reference's layouts (no host restatement).

        subdomains[tv]: nnodes (per level), free_dof (per level, increasing nodal dofs), K (per
        level, condensed consStif CSR), S (per level < L, scalar stencil CSR) -- or P (per level < L,
        the reference's condensed realProl, for rotated nodes) --, consForc, and optionally presc
        (3N nodal Dirichlet values), coords (N x 3) and hang = (nnodes_all, H): the hanging level
        (rows 3N.. of prolOper[maxiLeve], ddpca_problem_set_hanging).
        interfaces[ts]: body (2), fric, nip, nnc (2), pemaDiag, inpoNgap, ops[s][name] CSR for
        the names in Problem.IFACE_OPS.
        coarse (optional, the caller's MCONTACT::MULTISCALE_1 output, muscSett = 2): doleMcsc,
        baseReco, globCoup_1, globForc_1, globTran_1[ts][s], globTran_D_1[tv], accuProl[tv]; or
        its MULTISCALE output (muscSett = 1) with latin=True: doleMcsc, baseReco, globCoup,
        globTran / globTran_pena / globTran_D [ts][s], accuProl[tv]."""
        self = cls.__new__(cls)
        h = C.c_void_p()
        _check(lib().ddpca_problem_empty(len(subdomains), len(interfaces), C.byref(h)))
        self._h = h
        self.kind = "operators"
        keep = []

        def arr(a, dt):
            a = np.ascontiguousarray(a, dtype=dt)
            keep.append(a)
            return a

        def ptrs(lst, ctype):
            p = (C.c_void_p * max(1, len(lst)))(*[a.ctypes.data for a in lst])
            keep.append(p)
            return p

        for tv, s in enumerate(subdomains):
            nlev = len(s["nnodes"])
            K = [m.tocsr() for m in s["K"]]
            use_p = "P" in s
            S = [m.tocsr() for m in (s["P"] if use_p else s.get("S", []))]
            presc = s.get("presc")
            coords = s.get("coords")
            fn = lib().ddpca_problem_set_subdomain_prol if use_p else lib().ddpca_problem_set_subdomain
            _check(fn(
                self._h, tv, nlev, _ptr(arr(s["nnodes"], np.int64)), _ptr(arr([m.shape[0] for m in K], np.int64)),
                ptrs([arr(f, np.int32) for f in s["free_dof"]], None),
                ptrs([arr(m.indptr, np.int64) for m in K], None), ptrs([arr(m.indices, np.int32) for m in K], None),
                ptrs([arr(m.data, np.float64) for m in K], None),
                ptrs([arr(m.indptr, np.int64) for m in S], None), ptrs([arr(m.indices, np.int32) for m in S], None),
                ptrs([arr(m.data, np.float64) for m in S], None), _ptr(arr(s["consForc"], np.float64)),
                None if presc is None else _ptr(arr(presc, np.float64)),
                None if coords is None else _ptr(arr(np.asarray(coords).reshape(-1), np.float64))))
            if s.get("hang") is not None:
                n_all, Hm = s["hang"]
                Hm = Hm.tocsr()
                hv = _CsrArg(Hm.shape[0], Hm.shape[1], _ptr(arr(Hm.indptr, np.int64)), _ptr(arr(Hm.indices, np.int32)),
                             _ptr(arr(Hm.data, np.float64)))
                _check(lib().ddpca_problem_set_hanging(self._h, tv, int(n_all), C.byref(hv)))
        for ts, f in enumerate(interfaces):
            ops = (_CsrArg * 14)()
            for side in range(2):
                for k, name in enumerate(cls.IFACE_OPS):
                    m = f["ops"][side][name].tocsr()
                    ops[7 * side + k] = _CsrArg(m.shape[0], m.shape[1], _ptr(arr(m.indptr, np.int64)),
                                                _ptr(arr(m.indices, np.int32)), _ptr(arr(m.data, np.float64)))
            _check(lib().ddpca_problem_set_interface(
                self._h, ts, int(f["body"][0]), int(f["body"][1]), float(f["fric"]), int(f["nip"]), int(f["nnc"][0]),
                int(f["nnc"][1]), _ptr(arr(f["pemaDiag"], np.float64)), _ptr(arr(f["inpoNgap"], np.float64)), ops))
        if coarse is not None and coarse.get("latin", False):
            def csr_arg(m):
                m = m.tocsr()
                return _CsrArg(m.shape[0], m.shape[1], _ptr(arr(m.indptr, np.int64)), _ptr(arr(m.indices, np.int32)),
                               _ptr(arr(m.data, np.float64)))
            nint = len(interfaces)

            def sides(name):
                return (_CsrArg * max(1, 2 * nint))(*[csr_arg(coarse[name][ts][s]) for ts in range(nint)
                                                      for s in range(2)])
            ap = (_CsrArg * len(subdomains))(*[csr_arg(m) for m in coarse["accuProl"]])
            gc = csr_arg(coarse["globCoup"])
            _check(lib().ddpca_problem_set_coarse_latin(
                self._h, _ptr(arr(coarse["doleMcsc"], np.int64)), _ptr(arr(coarse["baseReco"], np.int64)), C.byref(gc),
                sides("globTran"), sides("globTran_pena"), sides("globTran_D"), ap))
        elif coarse is not None:
            def csr_arg(m):
                m = m.tocsr()
                return _CsrArg(m.shape[0], m.shape[1], _ptr(arr(m.indptr, np.int64)), _ptr(arr(m.indices, np.int32)),
                               _ptr(arr(m.data, np.float64)))
            nint = len(interfaces)
            gt = (_CsrArg * max(1, 2 * nint))(*[csr_arg(coarse["globTran_1"][ts][s]) for ts in range(nint) for s in range(2)])
            gd = (_CsrArg * len(subdomains))(*[csr_arg(m) for m in coarse["globTran_D_1"]])
            ap = (_CsrArg * len(subdomains))(*[csr_arg(m) for m in coarse["accuProl"]])
            gc = csr_arg(coarse["globCoup_1"])
            _check(lib().ddpca_problem_set_coarse_operators(
                self._h, 2, _ptr(arr(coarse["doleMcsc"], np.int64)), _ptr(arr(coarse["baseReco"], np.int64)),
                C.byref(gc), _ptr(arr(coarse["globForc_1"], np.float64)), gt, gd, ap))
        _check(lib().ddpca_problem_finalize(self._h))
        return self

    def export_operators(self) -> tuple:
        """(subdomains, interfaces) of an established problem in from_operators' format -- what a
        reference-side caller would hand over from its own MCONTACT after ESTABLISH."""
        import scipy.sparse as sp
        subs = []
        for tv in range(self.nsub):
            G = self.grid(tv)
            L = G.maxiLeve
            nn = [int(x) for x in self.array("leveCount", tv)]
            flag = G.consFlag
            S = [sp.csr_matrix((self.array("S:w", tv, l), self.array("S:col", tv, l), self.array("S:ptr", tv, l)),
                               shape=(nn[l + 1], nn[l])) for l in range(L)]
            presc = np.zeros(3 * nn[-1])
            presc[self.array("consDofv", tv)] = self.array("dispForc", tv)  # both in constrained-dof order
            subs.append(dict(nnodes=nn, free_dof=[np.flatnonzero(flag[: 3 * nn[l]]) for l in range(L + 1)],
                             K=[G.consStif(l) for l in range(L + 1)], S=S, consForc=G.consForc, presc=presc,
                             coords=G.nodeCoor))
        ifaces = []
        for ts in range(self.nint):
            fric = float(self.array("iface_param", ts)[0])
            ifaces.append(dict(body=[int(b) for b in self.array("iface_body", ts)], fric=fric,
                               nip=len(self.array("ip_w", ts)),
                               nnc=[len(self.array("nodeCont", 2 * ts + s)) for s in range(2)],
                               pemaDiag=self.array("pemaDiag", ts), inpoNgap=self.array("inpoNgap", ts),
                               ops=[{n: self.csr(n, 2 * ts + s) for n in self.IFACE_OPS} for s in range(2)]))
        return subs, ifaces


def contact_search(mast_xyz, mast_segm, mast_2d, slav_xyz, slav_segm, slav_2d, buck, maxiDist: float = 1.0e12) -> dict:
    """CSEARCH::BUCKET_SORT + CONTACT_SEARCH (CSEARCH.h:205-230, 777-817): integration points of
    the contact between master faces (mast_segm, 4 node ids each, coordinates mast_xyz by node id,
    2-D bucket coordinates mast_2d) and slave faces, in the reference's order.  Returns node
    (n, 2, 4), shap (n, 2, 4), basis (n, 3, 3), gap (n), w (n) -- Problem.set_ips' arguments."""
    def a(x, dt):
        return np.ascontiguousarray(x, dtype=dt)
    mx, sx = a(mast_xyz, np.float64).reshape(-1), a(slav_xyz, np.float64).reshape(-1)
    ms, ss = a(mast_segm, np.int64).reshape(-1), a(slav_segm, np.int64).reshape(-1)
    m2, s2 = a(mast_2d, np.float64).reshape(-1), a(slav_2d, np.float64).reshape(-1)
    bk = a(buck, np.int64)
    h = C.c_void_p()
    _check(lib().ddpca_contact_search(_ptr(mx), len(mx) // 3, _ptr(sx), len(sx) // 3, len(ms) // 4, _ptr(ms), _ptr(m2),
                                      len(ss) // 4, _ptr(ss), _ptr(s2), _ptr(bk), float(maxiDist), C.byref(h)))
    try:
        n = int(lib().ddpca_ips_count(h))
        out = dict(node=np.zeros((n, 2, 4), np.int64), shap=np.zeros((n, 2, 4)), basis=np.zeros((n, 3, 3)),
                   gap=np.zeros(n), w=np.zeros(n))
        if n:
            _check(lib().ddpca_ips_get(h, _ptr(out["node"]), _ptr(out["shap"]), _ptr(out["basis"]), _ptr(out["gap"]),
                                       _ptr(out["w"])))
        return out
    finally:
        lib().ddpca_ips_destroy(h)


class LAGRANGE:
    """MCONTACT::LAGRANGE (MCONTACT.h:2847-3701): dual mortar + semi-smooth Newton, every Newton
    step's condensed system solved on the device by MGPIS-preconditioned BiCGSTAB (precType 1) or
    diagonal-preconditioned BiCGSTAB (precType 2).  Inputs as LAGRANGE reads them from MCONTACT
    (include/ddpca_amd.h, ddpca_lagrange_*); ``from_problem`` takes them from a host Problem."""

    def __init__(self, nsub: int, nint: int):
        h = C.c_void_p()
        _check(lib().ddpca_lagrange_create(nsub, nint, C.byref(h)))
        self._h, self.nsub, self.nint, self._keep = h, nsub, nint, []

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.ddpca_lagrange_destroy(h)
            self._h = None

    def _arr(self, a, dt):
        a = np.ascontiguousarray(a, dtype=dt)
        self._keep.append(a)
        return a

    def _csr(self, m):
        m = m.tocsr()
        m.sort_indices()
        ptr, col, val = self._arr(m.indptr, np.int64), self._arr(m.indices, np.int32), self._arr(m.data, np.float64)
        return _CsrArg(m.shape[0], m.shape[1], ptr.ctypes.data, col.ctypes.data, val.ctypes.data)

    def set_subdomain(self, tv: int, nnodes, free_dof, K, P, consForc, nnodes_all: int, G, hanging=None):
        nlev = len(nnodes)
        fd = [self._arr(f, np.int32) for f in free_dof]
        fdp = (C.c_void_p * nlev)(*[f.ctypes.data for f in fd])
        Ka = (_CsrArg * nlev)(*[self._csr(k) for k in K])
        Pa = (_CsrArg * max(1, nlev - 1))(*[self._csr(q) for q in P])
        Ga = self._csr(G)
        hg = None if hanging is None else self._arr(hanging, np.uint8)
        _check(lib().ddpca_lagrange_set_subdomain(
            self._h, tv, nlev, _ptr(self._arr(nnodes, np.int64)), _ptr(self._arr([len(f) for f in fd], np.int64)),
            C.cast(fdp, C.c_void_p), Ka, Pa, _ptr(self._arr(consForc, np.float64)), int(nnodes_all), C.byref(Ga),
            None if hg is None else _ptr(hg)))
        return self

    def set_interface(self, ts: int, body, fric: float, node, shap, basis, gap, w):
        n = len(w)
        _check(lib().ddpca_lagrange_set_interface(
            self._h, ts, int(body[0]), int(body[1]), float(fric), n, _ptr(self._arr(node, np.int64)),
            _ptr(self._arr(shap, np.float64)), _ptr(self._arr(basis, np.float64)), _ptr(self._arr(gap, np.float64)),
            _ptr(self._arr(w, np.float64))))
        return self

    @classmethod
    def from_problem(cls, problem: "Problem") -> "LAGRANGE":
        """The inputs of an established host Problem (its MULTIGRID hierarchies and integration
        points; no hanging level, no rotations there: the node-id map is consOper^T)."""
        import scipy.sparse as sp
        lg = cls(problem.nsub, problem.nint)
        for tv in range(problem.nsub):
            g = problem.grid(tv)
            L = g.maxiLeve
            nn = [int(x) for x in problem.array("leveCount", tv)]
            flag = np.asarray(g.consFlag)
            fd = [np.flatnonzero(flag[: 3 * nn[l]]) for l in range(L + 1)]
            G = sp.csr_matrix((np.ones(len(fd[L])), (fd[L], np.arange(len(fd[L])))), shape=(3 * nn[L], len(fd[L])))
            lg.set_subdomain(tv, nn, fd, [g.consStif(l) for l in range(L + 1)], [g.realProl(l) for l in range(L)],
                             g.consForc, nn[L], G)
        for ts in range(problem.nint):
            lg.set_interface(ts, problem.array("iface_body", ts), float(problem.array("iface_param", ts)[0]),
                             problem.array("ip_node", ts), problem.array("ip_shap", ts), problem.array("ip_basis", ts),
                             problem.array("ip_gap", ts), problem.array("ip_w", ts))
        return lg

    def solve(self, precType: int = 1, device: int = 0, max_newton: int = 50, **opts) -> int:
        """Returns tc, the reference's "Converge after tc-th iteration"."""
        o = default_options(**opts)
        return int(_check(lib().ddpca_lagrange_solve(self._h, device, precType, C.byref(o), max_newton)))

    def get(self, what: str, index: int = 0) -> np.ndarray:
        n = _check(lib().ddpca_lagrange_get(self._h, what.encode(), index, None, 0))
        out = np.zeros(n)
        if n:
            _check(lib().ddpca_lagrange_get(self._h, what.encode(), index, _ptr(out), n))
        return out


class MULTIGRID:
    """Read-only view of one subdomain's operators (MULTIGRID.h public members)."""

    def __init__(self, problem: Problem, tv: int):
        self.problem = problem
        self.tv = tv

    @property
    def maxiLeve(self) -> int:
        return int(self.problem.array("maxiLeve", self.tv)[0])

    @property
    def nodeCoor(self) -> np.ndarray:
        return self.problem.array("coords", self.tv).reshape(-1, 3)

    @property
    def consFlag(self) -> np.ndarray:
        return self.problem.array("consFlag", self.tv)

    @property
    def consForc(self) -> np.ndarray:
        return self.problem.array("consForc", self.tv)

    def consStif(self, level: int):
        return self.problem.csr("K", self.tv, level)

    def realProl(self, level: int):
        return self.problem.csr("P", self.tv, level)

    def hangRows(self):
        """Rows of prolOper[maxiLeve] past the MGPIS fine level (the hanging level's values over the
        level-maxiLeve nodal vector, OUTP_SUB1, MULTIGRID.h:1279); 0 rows without a hanging level."""
        return self.problem.csr("H", self.tv, 0)

    def OUTP_SUB1(self, x: np.ndarray) -> np.ndarray:
        """Condensed solution -> nodal displacement (MULTIGRID.h:1263-1281; no rotations)."""
        flag = self.consFlag
        fi = self.problem.array("freeIndex", self.tv)
        u = np.zeros(len(flag))
        u[flag == 1] = x[fi[flag == 1]]
        return u


# ============================================================================ device MGPIS
class MGPIS:
    """Device multigrid-preconditioned CG for one subdomain (MGPIS.h:8-225)."""

    def __init__(self, handle: C.c_void_p):
        self._h = handle

    @classmethod
    def from_problem(cls, problem: Problem, tv: int = 0, device: int = 0, **opts) -> "MGPIS":
        h = C.c_void_p()
        o = default_options(**opts)
        _check(lib().ddpca_problem_mgpis(problem.handle, tv, device, C.byref(o), C.byref(h)))
        return cls(h)

    @classmethod
    def from_csr(cls, nnodes: Sequence[int], free_dof: Sequence[np.ndarray], K: Sequence, S: Sequence,
                 device: int = 0, **opts) -> "MGPIS":
        """Reference layout: consStif[l] (scipy CSR, condensed), free_dof[l], scalar stencils S[l]."""
        nlev = len(nnodes)
        keep = []

        def arr(a, dt):
            a = np.ascontiguousarray(a, dtype=dt)
            keep.append(a)
            return a.ctypes.data

        nn = arr(nnodes, np.int64)
        nf = arr([k.shape[0] for k in K], np.int64)
        fd = (C.c_void_p * nlev)(*[arr(f, np.int32) for f in free_dof])
        kp = (C.c_void_p * nlev)(*[arr(k.indptr, np.int64) for k in K])
        kc = (C.c_void_p * nlev)(*[arr(k.indices, np.int32) for k in K])
        kv = (C.c_void_p * nlev)(*[arr(k.data, np.float64) for k in K])
        ns = max(nlev - 1, 1)
        sp_ = (C.c_void_p * ns)(*[arr(s.indptr, np.int64) for s in S])
        sc_ = (C.c_void_p * ns)(*[arr(s.indices, np.int32) for s in S])
        sw_ = (C.c_void_p * ns)(*[arr(s.data, np.float64) for s in S])
        h = C.c_void_p()
        o = default_options(**opts)
        _check(lib().mgpis_gpu_create(device, nlev, C.c_void_p(nn), C.c_void_p(nf), fd, kp, kc, kv, sp_, sc_, sw_,
                                      C.byref(o), C.byref(h)))
        return cls(h)

    @classmethod
    def from_prol(cls, nnodes: Sequence[int], free_dof: Sequence[np.ndarray], K: Sequence, P: Sequence,
                  device: int = 0, **opts) -> "MGPIS":
        """The reference's own MGPIS members: consStif[l] and realProl[l] (scipy CSR, condensed,
        MGPIS.h:8-38), free_dof[l] = consOper[l]'s nodal dofs; realProl may carry rotated-node
        blocks (MULTIGRID.h:1141-1181)."""
        nlev = len(nnodes)
        keep = []

        def arr(a, dt):
            a = np.ascontiguousarray(a, dtype=dt)
            keep.append(a)
            return a.ctypes.data

        nn = arr(nnodes, np.int64)
        nf = arr([k.shape[0] for k in K], np.int64)
        fd = (C.c_void_p * nlev)(*[arr(f, np.int32) for f in free_dof])
        kp = (C.c_void_p * nlev)(*[arr(k.indptr, np.int64) for k in K])
        kc = (C.c_void_p * nlev)(*[arr(k.indices, np.int32) for k in K])
        kv = (C.c_void_p * nlev)(*[arr(k.data, np.float64) for k in K])
        ns = max(nlev - 1, 1)
        pp = (C.c_void_p * ns)(*[arr(q.indptr, np.int64) for q in P])
        pc = (C.c_void_p * ns)(*[arr(q.indices, np.int32) for q in P])
        pv = (C.c_void_p * ns)(*[arr(q.data, np.float64) for q in P])
        h = C.c_void_p()
        o = default_options(**opts)
        _check(lib().mgpis_gpu_create_prol(device, nlev, C.c_void_p(nn), C.c_void_p(nf), fd, kp, kc, kv, pp, pc, pv,
                                           C.byref(o), C.byref(h)))
        return cls(h)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.mgpis_gpu_destroy(h)
            self._h = None

    def info(self) -> dict:
        out = (C.c_int64 * 7)()
        _check(lib().mgpis_gpu_info(self._h, out))
        return dict(nlev=out[0], nfree=out[1], nnzb=out[2], chunks=out[3], omega=out[4] / 1e6, lmax=out[5] / 1e6,
                    device=out[6])

    def bench_spmv(self, variant: int = 0, reps: int = 20) -> tuple:
        """Diagnostic: (ms per launch, algorithmic bytes per launch) of a fine-level kernel variant."""
        ms, nbytes = C.c_double(), C.c_double()
        _check(lib().mgpis_gpu_bench_spmv(self._h, variant, reps, C.byref(ms), C.byref(nbytes)))
        return ms.value, nbytes.value

    def CG_SOLV(self, precSwit: int, totaForc: np.ndarray, rtol: float = 1e-14, maxit: Optional[int] = None):
        """Returns (x, iterations, recursive relative residual); reference defaults rtol=1e-14, maxit=n."""
        b = np.ascontiguousarray(totaForc, dtype=np.float64)
        x = np.zeros_like(b)
        it = C.c_int64()
        rr = C.c_double()
        _check(lib().mgpis_gpu_solve(self._h, _ptr(b), _ptr(x), precSwit, rtol, len(b) if maxit is None else maxit,
                                     C.byref(it), C.byref(rr)))
        return x, it.value, rr.value

    def MULT_SOLV(self, totaForc: np.ndarray, maxit: int = 10000):
        """MGPIS::MULT_SOLV (MGPIS.h:130-160) -> (x, iterNumb at exit, ||b - Kx|| / ||b||)."""
        b = np.ascontiguousarray(totaForc, dtype=np.float64)
        x = np.zeros_like(b)
        it, rr = C.c_int64(), C.c_double()
        _check(lib().mgpis_gpu_mult_solve(self._h, _ptr(b), _ptr(x), maxit, C.byref(it), C.byref(rr)))
        return x, it.value, rr.value

    def BiCGSTAB_SOLV(self, precSwit: int, totaForc: np.ndarray, rtol: float = 1e-14,
                      maxit: Optional[int] = None):
        """MGPIS::BiCGSTAB_SOLV (MGPIS.h:350-432) -> (x, iterNumb, recursive ||r|| / ||b||, breakdown)."""
        b = np.ascontiguousarray(totaForc, dtype=np.float64)
        x = np.zeros_like(b)
        it, rr, bd = C.c_int64(), C.c_double(), C.c_int()
        _check(lib().mgpis_gpu_bicgstab(self._h, _ptr(b), _ptr(x), precSwit, rtol,
                                        len(b) if maxit is None else maxit, C.byref(it), C.byref(rr), C.byref(bd)))
        return x, it.value, rr.value, bool(bd.value)

    def GMRES_SOLV(self, precSwit: int, totaForc: np.ndarray, rtol: float = 1e-12, maxit: Optional[int] = None,
                   restart: int = 10):
        """MGPIS::GMRES_SOLV (MGPIS.h:228-348) -> (x, iterNumb, true ||b - Kx|| / ||b||)."""
        b = np.ascontiguousarray(totaForc, dtype=np.float64)
        x = np.zeros_like(b)
        it, rr = C.c_int64(), C.c_double()
        _check(lib().mgpis_gpu_gmres(self._h, _ptr(b), _ptr(x), precSwit, rtol, len(b) if maxit is None else maxit,
                                     restart, C.byref(it), C.byref(rr)))
        return x, it.value, rr.value

    def MULT_VCYC(self, r: np.ndarray) -> np.ndarray:
        r = np.ascontiguousarray(r, dtype=np.float64)
        z = np.zeros_like(r)
        _check(lib().mgpis_gpu_vcycle(self._h, _ptr(r), _ptr(z)))
        return z

    def spmv(self, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros_like(x)
        info = self.info()
        _check(lib().mgpis_gpu_spmv(self._h, info["nlev"] - 1, _ptr(x), _ptr(y)))
        return y

    def spmv_vcycle_copy(self, x: np.ndarray) -> np.ndarray:
        """y = K x through the V-cycle's reduced-precision copy of the fine level (precond_fp32 >= 1)."""
        x = np.ascontiguousarray(x, dtype=np.float64)
        y = np.zeros_like(x)
        _check(lib().mgpis_gpu_spmv_copy(self._h, self.info()["nlev"] - 1, 1, _ptr(x), _ptr(y)))
        return y


# ============================================================================ device MCONTACT
def write_resuDisp(path: str, disp: np.ndarray, rot_node=None, rot=None) -> None:
    d = np.ascontiguousarray(disp, dtype=np.float64)
    rn = np.ascontiguousarray([] if rot_node is None else rot_node, dtype=np.int64)
    rm = np.ascontiguousarray(np.zeros((0, 9)) if rot is None else rot, dtype=np.float64).reshape(-1)
    _check(lib().ddpca_write_resuDisp(str(path).encode(), _ptr(d), len(d) // 3, len(rn), _ptr(rn), _ptr(rm)))


def write_resuCont(path: str, fric: float, gamma: np.ndarray, stat=None, basis=None) -> None:
    g = np.ascontiguousarray(gamma, dtype=np.float64)
    nip = len(g) if fric == 0.0 else len(g) // 3
    st = np.ascontiguousarray(np.zeros(nip) if stat is None else stat, dtype=np.int32)
    bs = np.ascontiguousarray(np.zeros(9 * nip) if basis is None else basis, dtype=np.float64).reshape(-1)
    _check(lib().ddpca_write_resuCont(str(path).encode(), fric, nip, _ptr(g), _ptr(st), _ptr(bs)))


def write_resuMoni(path: str, rows: np.ndarray) -> None:
    r = np.ascontiguousarray(np.atleast_2d(rows), dtype=np.float64)
    _check(lib().ddpca_write_resuMoni(str(path).encode(), _ptr(r), r.shape[0], r.shape[1]))


def mass_solve(systems: Sequence, b: np.ndarray, rtol: float = 1e-14, maxit: int = 2000, fuse_alpha: int = -1,
               device: int = 0):
    """The ADMM loop's batched surface-mass Jacobi-PCG on its own (ddpca_mass_solve): systems = square
    scipy CSR matrices, b their right-hand sides concatenated.  Returns (x, iterations per system);
    a breakdown raises DdpcaError(DDPCA_ENUMERIC) with the last good iterate in the .x attribute."""
    keep = []
    arr = (_CsrArg * len(systems))()
    for k, m in enumerate(systems):
        m = m.tocsr()
        ptr, col, val = (np.ascontiguousarray(m.indptr, np.int64), np.ascontiguousarray(m.indices, np.int32),
                         np.ascontiguousarray(m.data, np.float64))
        keep += [ptr, col, val]
        arr[k] = _CsrArg(m.shape[0], m.shape[1], ptr.ctypes.data, col.ctypes.data, val.ctypes.data)
    b = np.ascontiguousarray(b, dtype=np.float64)
    x = np.zeros_like(b)
    its = np.zeros(len(systems), np.int64)
    rc = lib().ddpca_mass_solve(device, len(systems), arr, _ptr(b), _ptr(x), rtol, maxit, fuse_alpha, _ptr(its))
    if rc < 0:
        e = DdpcaError(rc, lib().ddpca_last_error().decode())
        e.x, e.iters = x, its
        raise e
    return x, its


class MCONTACT:
    """Device ADMM loop of MCONTACT::CONTACT_ANALYSIS (MCONTACT.h:2493-2845) for one rank."""

    def __init__(self, problem: Problem, device: int = 0, rank: int = 0, nranks: int = 1,
                 owner: Optional[Sequence[int]] = None, **opts):
        nsub = problem.nsub
        own = np.zeros(nsub, np.int32) if owner is None else np.ascontiguousarray(owner, dtype=np.int32)
        self._owner = own
        h = C.c_void_p()
        o = default_options(**opts)
        _check(lib().mcontact_gpu_create(problem.handle, device, rank, nranks, _ptr(own), C.byref(o), C.byref(h)))
        self._h = h
        self.problem = problem
        self.nsub, self.nint = nsub, problem.nint

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and _lib is not None:
            _lib.mcontact_gpu_destroy(h)
            self._h = None

    @staticmethod
    def unique_id() -> bytes:
        buf = (C.c_char * 128)()
        _check(lib().mcontact_gpu_unique_id(buf))
        return bytes(buf)

    def comm_init(self, uid: bytes) -> None:
        buf = (C.c_char * 128).from_buffer_copy(uid)
        _check(lib().mcontact_gpu_comm_init(self._h, buf))

    @staticmethod
    def comm_local(ranks: Sequence["MCONTACT"]) -> None:
        """Connect the rank handles of ONE process (ranks[r] = rank r) through the in-process test
        transport (mcontact_gpu_comm_local); run each rank's CONTACT_ANALYSIS on its own thread."""
        arr = (C.c_void_p * len(ranks))(*[m._h.value for m in ranks])
        _check(lib().mcontact_gpu_comm_local(arr, len(ranks)))

    def comm_loopback(self) -> None:
        """Timing only (mcontact_gpu_comm_loopback): this rank alone on its GPU, every exchange
        returned to itself, all-reduces the identity; its problem must be established in full."""
        _check(lib().mcontact_gpu_comm_loopback(self._h, self.problem.handle))

    def comm_check(self, n: int = 1000) -> None:
        """Collective transport check (mcontact_gpu_comm_check): tagged messages to every rank and an
        all-reduce, every element exact; raises DdpcaError(DDPCA_ECOMM) otherwise."""
        _check(lib().mcontact_gpu_comm_check(self._h, int(n)))

    def CONTACT_ANALYSIS(self, maxit: int = 3000, check: bool = True) -> int:
        return _check(lib().mcontact_gpu_iterate(self._h, maxit, 1 if check else 0))

    def monitor(self) -> np.ndarray:
        ncol = 2 * self.nsub + 8 * self.nint + 2
        rows = _check(lib().mcontact_gpu_monitor(self._h, None, 0))
        out = np.zeros((rows, ncol))
        if rows:
            _check(lib().mcontact_gpu_monitor(self._h, out.ctypes.data_as(_DP), rows))
        return out

    def get(self, what: str, index: int = 0) -> np.ndarray:
        n = _check(lib().mcontact_gpu_get(self._h, what.encode(), index, None, 0))
        dtype = (np.int64 if what in ("pcg_iters", "owned", "mass_iters", "coarse_solve", "gs_rows")
                 else np.int32 if what == "fricStat" else np.float64)
        out = np.zeros(n, dtype)
        if n:
            _check(lib().mcontact_gpu_get(self._h, what.encode(), index, _ptr(out), n))
        return out

    # ---- result files in the reference's formats (host writers, include/ddpca_amd.h)
    def OUTP_SUB2(self, tv: int, path: str) -> None:
        """resuDisp_<tv>.txt of an owned subdomain (MULTIGRID::OUTP_SUB2, MULTIGRID.h:1288-1307)."""
        write_resuDisp(path, self.get("resuDisp", tv))

    def OUTPUT_PRTR(self, ts: int, path: str) -> None:
        """resuCont_<ts>.txt of an interface this rank handles (MCONTACT::OUTPUT_PRTR, MCONTACT.h:97-123)."""
        fric = float(self.problem.array("iface_param", ts)[0])
        write_resuCont(path, fric, self.get("inpoGamm", ts), self.get("fricStat", ts),
                       self.problem.array("ip_basis", ts))

    def write_resuMoni(self, path: str) -> None:
        """resuMoni.txt (MCONTACT.h:2502, 2742-2836): every MONITOR row recorded so far."""
        write_resuMoni(path, self.monitor())

    def timing(self) -> dict:
        out = (C.c_double * 10)()
        _check(lib().mcontact_gpu_timing(self._h, out))
        keys = ["total_ms", "solve_ms", "iface_ms", "comm_ms", "spmv_kernel_ms", "spmv_samples", "pcg_iterations",
                "spmv_bytes_per_launch", "dof_iterations", "owned_dofs"]
        return dict(zip(keys, list(out)))

    BYTE_PHASES = ("pcg_fine", "pcg_coarse", "coarse_space", "body_rhs", "interface", "mass_cg", "monitor")

    def bytes(self) -> dict:
        """Algorithmic HBM bytes of the last CONTACT_ANALYSIS call per phase (mcontact_gpu_bytes),
        plus the body-balance PCG's kernel launches."""
        out = (C.c_double * 8)()
        _check(lib().mcontact_gpu_bytes(self._h, out, 8))
        d = dict(zip(self.BYTE_PHASES, list(out)[:7]))
        d["pcg_launches"] = out[7]
        return d


__all__ = ["Problem", "MULTIGRID", "MGPIS", "MCONTACT", "DdpcaError", "lib", "gpu_available", "default_options",
           "contact_search", "mass_solve", "stream_ceiling", "probe_grid_barrier",
           "LIBPATH", "HEADLINE_OPTIONS", "HEADLINE_OPTIONS_SMALL", "headline_options", "HEADLINE_MUSC",
           "HEADLINE_WORKLOAD",
           "headline_problem"]
