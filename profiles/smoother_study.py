"""Smoother study on the headline's subdomain hierarchy (CPU, scipy): PCG iterations to the
reference's stop rule (||r|| <= 1e-14 ||b||, x0 = 0) with the V(1,1) preconditioners the device
could run at equal fine-level operator passes:

  bj     3x3 node-block Jacobi, damping 1.7 / lambda_max(D^-1 K) (the headline's smoother)
  mcgs   multicolour node-block Gauss-Seidel: forward over the colours before the coarse
         correction, backward after it (symmetric V-cycle); colours from a greedy colouring of
         the node graph (8 on a 27-point lattice)
  mcgs_fine  mcgs on the finest level only, bj below
  mcgs_coarse  bj on the finest level, mcgs below
  sgs    the reference's lexicographic point SGS (MGPIS.h:61-114) for comparison
  mcgs_band  (--general: bench.py's general mesh, contact band refined once more) mcgs on the finest
         level restricted to the band -- the rows of the nodes level L adds to level L-1 and their
         K_L neighbours -- bj below (level L-1 already smooths the unrefined rows' identical stencils)
  mcgs_band2 mcgs_band on the finest level and mcgs on level L-1, bj below; mcgs_two: mcgs on the two
         finest levels, bj below
  hgs_fine   hybrid (tile-local) multicolour GS on the finest level, bj below: the colours are swept
         inside 3D tiles of nodes (--tile tx,ty,tz, default 16,16,8), couplings across tiles read the
         values from before the sweep (block Jacobi over tiles, GS inside: what one launch per sweep
         with x in LDS would compute; symmetric, as the backward sweep is the forward one's adjoint)

    python profiles/smoother_study.py [gl] [subdomain]
"""
from __future__ import annotations

import importlib
import sys
import time
from pathlib import Path

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spl

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
D = importlib.import_module("ddpca-admm_amd")


TILE = (16, 16, 8)
RHS = None
NEWONLY = False  # --new-only: the band is the new nodes alone (no neighbour ring)
ORDER = None  # --order 0,7,...: the fine level's colours swept in this order (forward; backward reversed)


GENERAL = False


def hierarchy(gl: int, tv: int):
    P = D.headline_problem(gl=gl, **(D.GENERAL_FEATURES if GENERAL else {})).ESTABLISH()
    global COORD, NN
    COORD = np.asarray(P.array("coords", tv), dtype=np.float64).reshape(-1, 3)
    G = P.grid(tv)
    L = G.maxiLeve
    nn = [int(x) for x in P.array("leveCount", tv)]
    NN = nn
    flag = np.asarray(P.array("consFlag", tv))
    K = [G.consStif(l).tocsr() for l in range(L + 1)]
    Pr = [G.realProl(l).tocsr() for l in range(L)]
    node = []
    for l in range(L + 1):
        dofs = np.nonzero(flag[:3 * nn[l]])[0]
        assert len(dofs) == K[l].shape[0]
        node.append(dofs // 3)
    b = np.asarray(P.array("consForc", tv), dtype=np.float64)
    if RHS is not None:  # --rhs FILE.npy: a right-hand side saved by profiles/dump_rhs.py
        b = np.load(RHS)
        assert len(b) == K[L].shape[0]
    if not np.any(b):
        b = np.random.default_rng(0).standard_normal(K[L].shape[0])
    return K, Pr, node, b


class BlockDiag:
    """node blocks of K (1-3 free dofs per node) and their inverses, padded to 3x3"""

    def __init__(self, K, node):
        n = K.shape[0]
        un, first = np.unique(node, return_index=True)
        self.nodes = un
        self.loc = np.searchsorted(un, node)
        self.slot = np.arange(n) - first[self.loc]
        nb = len(un)
        Bk = np.zeros((nb, 3, 3))
        Kc = K.tocoo()
        same = self.loc[Kc.row] == self.loc[Kc.col]
        Bk[self.loc[Kc.row[same]], self.slot[Kc.row[same]], self.slot[Kc.col[same]]] = Kc.data[same]
        for k in range(3):
            pad = Bk[:, k, k] == 0
            Bk[pad, k, k] = 1.0
        self.inv = np.linalg.inv(Bk)
        self.n = n

    def apply(self, r, rows=None):
        rows = np.arange(self.n) if rows is None else rows
        v = np.zeros((self.inv.shape[0], 3))
        v[self.loc[rows], self.slot[rows]] = r
        w = np.einsum("nij,nj->ni", self.inv, v)
        return w[self.loc[rows], self.slot[rows]]


def colouring(K, node):
    """greedy colouring of the node graph in node order"""
    bd_loc = np.unique(node, return_inverse=True)[1]
    nb = bd_loc.max() + 1
    A = sp.csr_matrix((np.ones(K.nnz), K.indices, K.indptr), shape=K.shape)
    R = sp.csr_matrix((np.ones(len(node)), (bd_loc, np.arange(len(node)))), shape=(nb, len(node)))
    G = (R @ A @ R.T).tocsr()
    col = -np.ones(nb, dtype=np.int64)
    for v in range(nb):
        nb_cols = col[G.indices[G.indptr[v]:G.indptr[v + 1]]]
        used = set(nb_cols[nb_cols >= 0].tolist())
        c = 0
        while c in used:
            c += 1
        col[v] = c
    return col[bd_loc]


class VCycle:
    def __init__(self, K, Pr, node, smoother: str, coarse: int = 0):
        # "name" or "name:nu_fine:nu_coarse" (sweeps before and after the coarse correction)
        smoother, *nus = smoother.split(":")
        # "name@w": over-relaxed multicolour sweeps (SSOR-type: the same w forward and backward)
        smoother, _, w = smoother.partition("@")
        self.w = float(w) if w else 1.0
        self.nu_fine, self.nu_coarse = (int(nus[0]), int(nus[1])) if nus else (1, 1)
        self.nu_second = int(nus[2]) if len(nus) > 2 else self.nu_coarse  # level L-1
        self.K, self.Pr, self.sm = K, Pr, smoother
        self.L = len(K) - 1
        self.coarse = coarse
        self.lu = spl.splu(K[coarse].tocsc())
        self.bd, self.omega, self.rows, self.Krows, self.tri = {}, {}, {}, {}, {}
        for l in range(coarse + 1, self.L + 1):
            bd = BlockDiag(K[l], node[l])
            self.bd[l] = bd
            if self.is_bj(l):
                lam = spl.eigsh(spl.LinearOperator(K[l].shape, matvec=lambda x, l=l: bd.apply(K[l] @ x)), k=1,
                                which="LM", return_eigenvectors=False, tol=1e-3)[0]
                self.omega[l] = 1.7 / lam
            elif smoother.startswith("mcgs") or smoother.startswith("hgs") or smoother.startswith("bmcgs"):
                c = colouring(K[l], node[l])
                if smoother.startswith("bmcgs") and l == self.L:
                    # 2x2x2 node blocks coloured by the block lattice's parity, each block swept in
                    # lexicographic order: 64 "colours" = block colour x position in the block
                    xyz = COORD[node[l]]
                    idx = []
                    for d in range(3):
                        u = np.unique(np.round(COORD[np.unique(node[l])][:, d], 12))
                        idx.append(np.searchsorted(u, np.round(xyz[:, d], 12)))
                    bx, by, bz = idx[0] // 2, idx[1] // 2, idx[2] // 2
                    bc = (bx % 2) + 2 * (by % 2) + 4 * (bz % 2)
                    lp = (idx[0] % 2) + 2 * (idx[1] % 2) + 4 * (idx[2] % 2)
                    c = bc * 8 + lp
                order = ORDER if ORDER and l == self.L and len(ORDER) == c.max() + 1 else list(range(c.max() + 1))
                self.rows[l] = [np.nonzero(c == k)[0] for k in order]
                if smoother in ("mcgs_band", "mcgs_band2") and l == self.L:
                    new = (node[l] >= NN[l - 1]).astype(np.float64)
                    A = sp.csr_matrix((np.ones(K[l].nnz), K[l].indices, K[l].indptr), shape=K[l].shape)
                    band = (new > 0) | ((A @ new) > 0) if not NEWONLY else new > 0
                    self.band_rows = int(band.sum())
                    self.rows[l] = [r[band[r]] for r in self.rows[l]]
                self.Krows[l] = [K[l][r] for r in self.rows[l]]
                if smoother.startswith("hgs"):
                    # tile of every dof: 3D blocks of TILE nodes on the level's node lattice
                    xyz = COORD[node[l]]
                    tid = np.zeros(len(xyz), dtype=np.int64)
                    for d in range(3):
                        u = np.unique(np.round(COORD[np.unique(node[l])][:, d], 12))
                        idx = np.searchsorted(u, np.round(xyz[:, d], 12))
                        tid = tid * (len(u) // TILE[d] + 2) + idx // TILE[d]
                    self.split = getattr(self, "split", {})
                    sp_l = []
                    for r, Kr in zip(self.rows[l], self.Krows[l]):
                        Kc = Kr.tocoo()
                        same = tid[r][Kc.row] == tid[Kc.col]
                        Kin = sp.csr_matrix((Kc.data[same], (Kc.row[same], Kc.col[same])), shape=Kr.shape)
                        Koff = sp.csr_matrix((Kc.data[~same], (Kc.row[~same], Kc.col[~same])), shape=Kr.shape)
                        sp_l.append((Kin, Koff))
                    self.split[l] = sp_l
                    self.ntile = len(np.unique(tid))
                    if "l1" in smoother:
                        # l1 hybrid GS (Baker, Falgout, Kolev, Yang 2011): each row's diagonal gets the
                        # absolute sum of its off-tile couplings, which makes the tile-Jacobi smoother
                        # convergent whatever the coupling
                        Kc = K[l].tocoo()
                        off = tid[Kc.row] != tid[Kc.col]
                        l1 = np.bincount(Kc.row[off], weights=np.abs(Kc.data[off]), minlength=K[l].shape[0])
                        self.bd[l] = BlockDiag(K[l] + sp.diags(l1), node[l])
            elif smoother.startswith("sgs"):
                self.tri[l] = (sp.tril(K[l], format="csr"), sp.triu(K[l], format="csr"))

    def is_bj(self, l):
        return self.sm == "bj" or (self.sm in ("mcgs_fine", "hgs_fine", "hgs_l1_fine", "mcgs_band", "bmcgs_fine", "mcgs_ssor_fine") and l < self.L) or \
            (self.sm in ("mcgs_band2", "mcgs_two", "mcgs_l1ssor") and l < self.L - 1) or \
            (self.sm == "mcgs_coarse" and l == self.L)

    def smooth(self, l, x, b, forward: bool):
        K = self.K[l]
        if self.is_bj(l):
            return x + self.omega[l] * self.bd[l].apply(b - K @ x)
        if self.sm.startswith("hgs"):
            order = range(len(self.rows[l])) if forward else reversed(range(len(self.rows[l])))
            x0, x = x, x.copy()
            for k in order:
                r = self.rows[l][k]
                Kin, Koff = self.split[l][k]
                x[r] += self.bd[l].apply(b[r] - Kin @ x - Koff @ x0, r)
            return x
        if self.sm.startswith("mcgs") or self.sm.startswith("bmcgs"):
            order = range(len(self.rows[l])) if forward else reversed(range(len(self.rows[l])))
            x = x.copy()
            for k in order:
                r = self.rows[l][k]
                x[r] += self.w * self.bd[l].apply(b[r] - self.Krows[l][k] @ x, r)
            return x
        lo, up = self.tri[l]
        if forward:
            return x + spl.spsolve_triangular(lo, b - K @ x, lower=True)
        return x + spl.spsolve_triangular(up, b - K @ x, lower=False)

    def apply(self, l, b):
        if l == self.coarse:
            return self.lu.solve(b)
        nu = self.nu_fine if l == self.L else self.nu_second if l == self.L - 1 else self.nu_coarse
        # SSOR smoothing ("ssor" in the name, the reference's MULT_VCYC, MGPIS.h:64-76, 101-114):
        # every smoothing step is a forward AND a backward sweep, before and after the coarse
        # correction, on the levels the named smoother sweeps
        ssor = "ssor" in self.sm and not self.is_bj(l)
        if self.sm == "mcgs_l1ssor":  # colour GS on the fine level, colour SSOR on L-1, bj below
            ssor = l == self.L - 1
        x = np.zeros_like(b)
        for _ in range(nu):
            x = self.smooth(l, x, b, True)
            if ssor:
                x = self.smooth(l, x, b, False)
        r = b - self.K[l] @ x
        x = x + self.Pr[l - 1] @ self.apply(l - 1, self.Pr[l - 1].T @ r)
        for _ in range(nu):
            if ssor:
                x = self.smooth(l, x, b, True)
            x = self.smooth(l, x, b, False)
        return x


def pcg(K, b, M, rtol=1e-14, maxit=500):
    x = np.zeros_like(b)
    r = b.copy()
    z = M(r)
    p = z.copy()
    rz = r @ z
    nb = np.linalg.norm(b)
    for it in range(1, maxit + 1):
        q = K @ p
        a = rz / (p @ q)
        x += a * p
        r -= a * q
        if np.linalg.norm(r) <= rtol * nb:
            return it, x
        z = M(r)
        rz, rz0 = r @ z, rz
        p = z + (rz / rz0) * p
    return maxit, x


def round_h16(K, node):
    """K with every 3x3 node block stored as 2^e x nine fp16 values (the device's block-exponent
    fp16 copy of the fine level, precond_fp32 = 2)"""
    Kc = K.tocoo()
    key = node[Kc.row].astype(np.int64) * (node.max() + 1) + node[Kc.col]
    uk, inv = np.unique(key, return_inverse=True)
    mx = np.zeros(len(uk))
    np.maximum.at(mx, inv, np.abs(Kc.data))
    _, e = np.frexp(mx)
    sc = np.ldexp(1.0, e)[inv]
    v = (Kc.data / sc).astype(np.float16).astype(np.float64) * sc
    return sp.csr_matrix((v, (Kc.row, Kc.col)), shape=K.shape)


QSCALE = "pow2"  # --qscale pow2 | exact | row (per block row, pow2)


def round_i8(K, node, bits=8):
    """K with every 3x3 node block stored as 2^e x nine signed (bits)-bit integers (a block-scaled
    integer copy: |q| <= 2^(bits-1) - 1, e the smallest exponent that fits the block's largest entry);
    --qscale exact: scale = max / qmax (not a power of two), row: one power-of-two scale per block row"""
    Kc = K.tocoo()
    key = node[Kc.row].astype(np.int64) * (node.max() + 1) + node[Kc.col]
    if QSCALE == "row":
        key = key * 3 + (Kc.row - np.searchsorted(node, node[Kc.row]))  # dof slot of the row within its node
    uk, inv = np.unique(key, return_inverse=True)
    mx = np.zeros(len(uk))
    np.maximum.at(mx, inv, np.abs(Kc.data))
    qmax = 2 ** (bits - 1) - 1
    if QSCALE == "exact":
        sc = (np.maximum(mx, 1e-300) / qmax)[inv]
    elif QSCALE.startswith("m"):  # scale 2^e (1 + k / 2^M), the smallest such that max / scale <= qmax
        M = int(QSCALE[1:])
        t = np.maximum(mx, 1e-300) / qmax
        e = np.floor(np.log2(t))
        k = np.ceil((t / np.ldexp(1.0, e.astype(np.int64)) - 1.0) * 2 ** M)
        sc = (np.ldexp(1.0, e.astype(np.int64)) * (1.0 + k / 2 ** M))[inv]
        lm = np.log2(np.maximum(mx, 1e-300) / mx.max())
        print(f"  block maxima below the level maximum: 2^-16 {np.mean(lm < -16):.2e}, 2^-24 {np.mean(lm < -24):.2e}, "
              f"2^-31 {np.mean(lm < -31):.2e} (nonzero blocks {np.sum(mx > 0)})")
    else:
        e = np.ceil(np.log2(np.maximum(mx, 1e-300) / qmax))
        sc = np.ldexp(1.0, e.astype(np.int64))[inv]
    v = np.clip(np.rint(Kc.data / sc), -qmax, qmax) * sc
    return sp.csr_matrix((v, (Kc.row, Kc.col)), shape=K.shape)


def main():
    global TILE, GENERAL, ORDER, NEWONLY, RHS, QSCALE
    if "--qscale" in sys.argv:
        QSCALE = sys.argv[sys.argv.index("--qscale") + 1]
    if "--rhs" in sys.argv:
        RHS = sys.argv[sys.argv.index("--rhs") + 1]
    GENERAL = "--general" in sys.argv
    NEWONLY = "--new-only" in sys.argv
    if "--order" in sys.argv:
        ORDER = [int(v) for v in sys.argv[sys.argv.index("--order") + 1].split(",")]
    if "--tile" in sys.argv:
        TILE = tuple(int(v) for v in sys.argv[sys.argv.index("--tile") + 1].split(","))
    gl = int(sys.argv[1]) if len(sys.argv) > 1 else 4
    tv = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    K, Pr, node, b = hierarchy(gl, tv)
    if "--h16" in sys.argv:
        # the V-cycle's fine level on the fp16 copy (the Krylov operator stays fp64)
        K16 = round_h16(K[-1], node[-1])
        Kv = K[:-1] + [K16]
        print("fine level rounded to block-exponent fp16: |K16 - K| / |K| =",
              spl.norm(K16 - K[-1]) / spl.norm(K[-1]))
    elif "--i8" in sys.argv or "--ibits" in sys.argv:
        # the V-cycle's finest levels on a block-scaled integer copy (--ibits B, default 8; --ilevels N
        # finest levels, default 1)
        bits = int(sys.argv[sys.argv.index("--ibits") + 1]) if "--ibits" in sys.argv else 8
        nl = int(sys.argv[sys.argv.index("--ilevels") + 1]) if "--ilevels" in sys.argv else 1
        Kv = list(K)
        for l in range(len(K) - nl, len(K)):
            Kv[l] = round_i8(K[l], node[l], bits)
            print(f"level {l} rounded to block-scaled int{bits}: |Kq - K| / |K| =",
                  spl.norm(Kv[l] - K[l]) / spl.norm(K[l]))
    else:
        Kv = K
    print(f"gl {gl} subdomain {tv}: levels {len(K)}, fine rows {K[-1].shape[0]}")
    for sm in sys.argv[3].split(",") if len(sys.argv) > 3 and not sys.argv[3].startswith("-") else ("bj", "mcgs", "mcgs_fine", "sgs"):
        t = time.time()
        V = VCycle(Kv, Pr, node, sm)
        it, x = pcg(K[-1], b, lambda r: V.apply(V.L, r))
        res = np.linalg.norm(b - K[-1] @ x) / np.linalg.norm(b)
        ncol = max((len(v) for v in V.rows.values()), default=0)
        extra = f"  tiles {V.ntile} of {TILE}" if sm.startswith("hgs") else \
            f"  band rows {V.band_rows} of {K[-1].shape[0]}" if sm.startswith("mcgs_band") else ""
        print(f"{sm:5s} PCG iterations {it:3d}  true relres {res:.2e}  colours {ncol}{extra}  ({time.time() - t:.1f} s)")


if __name__ == "__main__":
    main()
