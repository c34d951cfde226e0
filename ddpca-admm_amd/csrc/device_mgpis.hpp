// MGPIS on the GPU: multigrid-preconditioned CG (MGPIS.h:163-225) with a V-cycle
// (MGPIS.h:55-128) whose smoother is (block-)Jacobi or Chebyshev, built for gfx950.
//
// One MgpisDevice solves a BATCH of independent subdomains (every subdomain a rank owns) with
// one stream and one hipGraph: level l of all subdomains is concatenated, each subdomain padded
// to a multiple of 64 nodes so a 64-node chunk (= one wavefront) never straddles two of them.
// Every launch therefore covers all subdomains -- the coarse levels (a few thousand nodes per
// subdomain) get batch-wide grids instead of 8 latency-bound launches on 4 hardware queues --
// while the PCG scalars, stop flags, smoother coefficients and coarse inverses stay per
// subdomain (a converged subdomain's chunks exit at their first instruction).
//
// Node numbering: the reference numbers nodes level by level (a coarse level is a prefix of the
// next, MULTIGRID.h:884-910), which scatters a fine node's neighbours over the whole vector.  On
// the device every level >= 1 of every subdomain is renumbered lexicographically by (z, y, x)
// when coordinates are supplied, and each row's blocks are sorted by the new column: the 64
// lanes of a chunk then gather x from a few contiguous runs (measured bound: coalesced gathers
// take the fine SpMV from 5.4 to 6.7 TB/s).  The transfer operators are explicit index lists,
// so nothing depends on the prefix property; level 0 keeps the reference order.
//
// Layout in HBM (per level l, nodes in the device order inside each subdomain):
//   K  : SELL-64 over 3x3 blocks ("SELL-BSR3"): chunk = 64 consecutive node rows = one
//        wavefront, lane = node row; slot k of chunk c holds one block per lane:
//          col[(off[c]+k)*64 + lane]            int32 block column (batch-global node index)
//          val[((off[c]+k)*9 + ij)*64 + lane]   fp64, ij = 3*a + b of the 3x3 block
//        so every load of a slot is a contiguous 256 B (col) / 512 B (val) wave access.
//        Constrained dofs are kept in place with identity rows/cols (mask), which is the
//        reference's condensed operator consOper*K*consOper^T (MULTIGRID.h:1227) embedded
//        in the nodal space -- the 3x3 block structure survives Dirichlet condensation.
//   P  : scalar stencil (x) I3, fine-major (<= 8 parents, slot-major; a node also present on
//        the coarse level has itself as the only parent, weight 1) for prolongation and
//        coarse-major child lists (self first, weight 1) for restriction: gathers, no atomics.
//   A0^-1 : dense inverse of each subdomain's coarsest level (exact coarse solve, one GEMV).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

#include "../../include/ddpca_amd.h"
#include "device_common.hpp"
#include "sparse.hpp"

namespace ddpca {

// Storage type of streamed operator values (arithmetic is fp64 throughout).
enum ValType { kVal64 = 0, kVal32 = 1, kValH16 = 2, kValQ8 = 3 };  // H16: block-exponent fp16, Q8: block-scaled int8

// Per-subdomain scalar block of the PCG recurrence (device memory, read by every kernel).
struct PcgScal {
    double delta;     // r^T z
    double alpha, beta;
    double rr;        // ||r||^2
    double tol2;      // (rtol ||b||)^2
    double pq;        // p^T q
    double bb;        // ||b||^2
    int64_t iter;
    int64_t maxit;
    int done;         // set on convergence / cap / breakdown
    int fail;         // 1: NaN/Inf or non-positive curvature
};

// Operators of one subdomain, in the host (MULTIGRID restatement) layout.
struct SubdomainOps {
    std::vector<int64_t> nnodes;           // nodes of level <= l
    std::vector<const Bsr3*> K;            // unconstrained Galerkin operator per level
    const uint8_t* dof_free = nullptr;     // 3 * nnodes.back() flags (consFlag)
    // optional per-level flags (3 * nnodes[l] each) where a dof's status differs between levels
    // (LATIN's DOUBLE_M: a coarse contact node its finer level does not carry is a masked copy
    // there); empty = the fine flags' prefix on every level (consOper, MULTIGRID.h:1186-1243)
    std::vector<const uint8_t*> dof_free_lev;
    const uint8_t* free_flags(int l) const { return dof_free_lev.empty() ? dof_free : dof_free_lev[l]; }
    std::vector<const Stencil*> S;         // scalar prolongation stencils, nlev - 1
    const double* coords = nullptr;        // optional 3 * nnodes.back() node coordinates: when
                                           // given, levels >= 1 are renumbered on the device
};

struct LevelDev {
    int64_t nn = 0, nch = 0, nslots = 0, nnzb = 0;  // batch totals (nn, nch padded)
    std::vector<int64_t> noff, nloc, nnzb_sub;      // per subdomain: first node, real nodes, blocks
    DevBuf<int32_t> slots, col, csub;               // csub: chunk -> subdomain
    DevBuf<int16_t> col16;  // col - row node when every offset of the level fits 16 bits (else empty)
    DevBuf<int64_t> off;
    DevBuf<double> val;    // fp64 operator: fine level (Krylov operator), or every level when the
                           // V-cycle runs on fp64 operators
    DevBuf<float> val32;   // V-cycle operator rounded once to fp32 (opt.precond_fp32), levels >= 1
    DevBuf<uint16_t> val16;  // fine level's V-cycle copy in block-exponent fp16 (opt.precond_fp32 = 2)
    DevBuf<uint8_t> val8;    // ... in block-scaled int8 (opt.precond_fp32 = 3)
    // table mode: rows whose block values (in device slot order, masks applied) are bit-identical
    // share one table row; the kernel streams only column indices and a row type, the values
    // come from the cache-resident table (structured meshes: ~30x fewer distinct rows than rows)
    bool tbl = false;
    int64_t tstride = 0;     // doubles per table row (max row length * 9)
    int64_t ntypes = 0;
    int64_t nuniform = 0;    // chunks whose rows all share one type
    DevBuf<int32_t> rtype;   // per node row
    DevBuf<int32_t> ctype;   // per chunk: the common type, -1 = mixed
    DevBuf<double> tab;

    DevBuf<double> minv;   // point: 3 per node; block: 9 per node
    DevBuf<float> minv32;  // the same in fp32 (symmetrised) on reduced-precision levels
    DevBuf<double> dinv;   // point Jacobi inverse (diagonal preconditioner at the fine level)
    DevBuf<uint8_t> mask;  // bit a set = dof 3i+a free
    DevBuf<double> coef;   // [(sweep * nsub + sub) * 2 + {0,1}]: Chebyshev (c1, c2) / Jacobi (-, omega)
    std::vector<double> lmax;  // per subdomain, lambda_max(M K)
    // transfer from level l-1 (batch-global indices)
    std::vector<int64_t> tent_sub, tblk_sub;  // per subdomain: scalar stencil entries, 3x3 block entries
    DevBuf<int32_t> ppar;  // 8 x nn, slot-major, -1 = unused
    DevBuf<double> pw;     // weights (empty when uw)
    bool uw = false;       // uniform averaging: prolongation weight = 1 / parent count (nested
                           // refinement), computed in k_prolong instead of read
    // restriction: SELL-64 over the coarse nodes of level l-1 (chunk = 64 coarse nodes, lane =
    // node, slot k = k-th child: own fine copy first, padding = weight 0)
    DevBuf<int32_t> rslots;  // per coarse chunk
    DevBuf<int64_t> roff;    // per coarse chunk + 1
    DevBuf<int32_t> rcol;    // fine node
    DevBuf<double> rwt;
    // lattice transfers (uniform averaging on a lexicographically numbered box lattice, detected
    // at create, off with DDPCA_LATTICE=0): a fine node's parents are p0 + subset sums of three
    // coarse strides, a coarse node's children its fine copy f0 + sum d_k t_k (d in {-1,0,1}^3)
    // with weight 2^-|d|; the kernels compute the indices instead of streaming ppar / rcol / rwt
    bool lat = false;
    DevBuf<uint32_t> ppk;   // per fine node: p0 | (stride-subset code << 29)
    DevBuf<int32_t> pstr;   // per subdomain: 3 coarse strides
    DevBuf<uint32_t> rmsk;  // per coarse node: 27-bit mask of the children present, bit (d0+1) + 3(d1+1) + 9(d2+1)
    DevBuf<int32_t> rf0;    // per coarse node: its fine copy
    DevBuf<int32_t> rstr;   // per subdomain: 3 fine strides
    // block transfer entries (nodal rotations, MULTIGRID.h:1141-1181): P = S (x) I3 + sum of
    // 3x3 blocks, as CSR over the fine nodes that own one (prolongation) and over the coarse
    // nodes that receive one (restriction, B^T); nrot = 0 on plain S (x) I3 transfers
    int64_t nrot = 0, nrotc = 0;
    DevBuf<int32_t> rot_row, rot_par, rotc_row, rotc_kid;
    DevBuf<int64_t> rot_ptr, rotc_ptr;
    DevBuf<double> rot_blk, rotc_blk;
    // vectors (3 nn)
    DevBuf<double> x, t, b, r, d;
    // fp32 iterate copies (x0, x1, x2, 0 per node) of a block-Jacobi level, or empty
    // (precond_fp32 = 4, MgpisDevice constructor): the V-cycle's x / t pair in 16 B per node
    DevBuf<float> x4a, x4b;
};

// Multicolour node-block Gauss-Seidel on the fine level (opt.smoother = 3): the fine nodes of
// each member are coloured greedily in device order (8 colours on a 27-point lattice), each
// colour's rows packed into 64-row chunks of their own.  A chunk's off-diagonal blocks are split
// by the column's colour into L (earlier colours) and U (later colours), both in the V-cycle
// copy's storage type, columns as in the level's SELL (offsets from the row node or int32).
// The pre-smoothing forward sweep from a zero guess reads only L (x_i = M_i (b_i - L_i x),
// colour by colour); the residual after it is r_i = -U_i x exactly (the row's own equation is
// met), so sweep + residual cost one operator pass; the backward post-smoothing sweep reads L
// and U.  With the symmetrised M the V-cycle stays symmetric (pre = forward, post = backward).
struct GsFine {
    int ncol = 0;                        // colours
    int64_t nchunk = 0;                  // colour chunks of the batch, member-major, colour-minor
    std::vector<int64_t> first, count;   // per colour: its chunk ids in `list`
    DevBuf<int32_t> list;                // chunk ids grouped by colour
    DevBuf<int32_t> rowidx;              // per chunk lane: device row, ~first row of the chunk on pad lanes
    DevBuf<int32_t> csub, nsl, nsu;      // per chunk: member, L slots, U slots
    DevBuf<int64_t> offl, offu;          // per chunk: first L / U slot
    DevBuf<int32_t> col;                 // per slot lane (when the level has no 16-bit offsets)
    DevBuf<int16_t> col16;
    DevBuf<uint16_t> val16;
    DevBuf<uint8_t> val8;
    DevBuf<float> val32;
    DevBuf<double> val64;
    DevBuf<float> minvc;                 // the rows' fp32 3x3 inverses in chunk order, [chunk][ij][lane]
                                         // (coalesced; the natural array at stride 2 nodes wastes half of every line)
    DevBuf<int64_t> cb;                  // per member: first colour chunk (nsub + 1), the dot partials
    // precond_fp32 = 4: the sweeps' iterate as an fp32 copy, 16 B per node (x0, x1, x2, 0), which every
    // sweep gathers with one 16-B load per neighbour block instead of three 8-B fp64 loads; the
    // forward sweep and the prolongation write only it, the backward sweep also the fp64 output z.
    // The block products, the epilogues and z stay fp64: the preconditioner moves by the fp32
    // rounding of the neighbours' values (lattice fine transfers without block entries, no band)
    DevBuf<float> x4;
    DevBuf<double> w;  // colour SSOR (opt.smoother = 4, k_gs_ssor): the partial sums handed between sweeps
    DevBuf<float> r4;  // ... and the residual after the forward sweep (PH 1), which the fine restriction reads
    DevBuf<double> partial;              // per colour chunk: the backward sweep's dot partials (their own
                                         // buffer: a split batch's other half writes the Krylov partials meanwhile)
    std::vector<int64_t> nnzb_sub;       // per member: stored off-diagonal blocks (byte model)
    std::vector<int64_t> slots_sub;      // per member: L + U slots incl. padding
    // algorithmic bytes of each launch over the whole batch, in launch order: forward colours
    // 0..K-1, the residual, backward colours K-1..0 (stored blocks, per-row vectors, every distinct
    // x entry gathered once; profiles/gs_table.py sets the rocprof / PMC figures beside them)
    std::vector<double> launch_bytes;
    std::vector<double> gx_f, gx_b, rows_k;  // per colour: distinct x gathered (forward, backward), rows
    double gx_r = 0.0;                       // distinct x the residual gathers
    std::vector<double> gx_u, nl_k, nu_k;    // per colour: distinct U-side x gathered, L / U blocks
    double gx_l = 0.0, vb = 0.0;             // distinct L-side x over all colours; bytes per stored block
    // band mode (locally refined fine level): the colours cover only the band -- the
    // nodes the fine level adds to the next coarser one and their neighbours; two more chunk groups
    // per member follow the colours: the ring (non-band rows with a band neighbour: their band
    // columns only, for the residual) and the far rows (no blocks).  first / count then hold ncol + 2
    // groups; the sweeps run over the colours, k_gs_aux over the ring and far groups.
    bool band = false;
    std::vector<int64_t> band_rows_sub, ring_rows_sub, far_rows_sub, ring_nnzb_sub;
};

class MgpisDevice {
public:
    // general: the operators may be nonsymmetric (LAGRANGE's condensed systems under Coulomb
    // friction): LU coarse inverse, no symmetrised fp32 smoother copy
    // diag_only: a handle for the diagonal-preconditioned drivers only (no dense coarse inverse)
    MgpisDevice(int device, const std::vector<SubdomainOps>& subs, const mgpis_options_t& opt, bool general = false,
                bool diag_only = false);
    bool general = false;
    bool no_coarse = false;  // one-level handle without the dense inverse (diagonal drivers only)
    // per subdomain's dense coarse inverse: kind 0 SPD potri, 1 LU (getri, residual checked),
    // 2 SVD pseudo-inverse; the LU's ||A^-1 A - I||_inf (INFINITY when its pivots failed); the
    // singular values the pseudo-inverse dropped
    struct CoarseInverse {
        int kind;
        double resid;
        int64_t dropped;
    };
    std::vector<CoarseInverse> coarse_inverse;
    ~MgpisDevice();

    int device = 0;
    int nsub = 0;
    hipStream_t stream = nullptr;
    mgpis_options_t opt{};
    std::vector<LevelDev> lev;
    GsFine gs;                            // opt.smoother = 3: the fine level's colour structure
    bool gs_fine() const { return gs.ncol > 0; }
    // chunk partials the V-cycle's dot product leaves and their bounds (k_fin after vcycle(dot))
    const int64_t* vc_cb() const { return gs_fine() ? gs.cb.p : fin_cb.p; }
    double* vc_partial() const { return gs_fine() ? gs.partial.p : partial.p; }
    // exact coarse solve on level clev: per-subdomain dense inverses, packed
    int clev = 0;
    DevBuf<double> ainv;
    DevBuf<float> ainv32;      // the same in fp32 (reduced-precision preconditioner storage)
    DevBuf<int64_t> aoff;      // per subdomain offset into ainv
    DevBuf<int64_t> c_noff;    // per subdomain first node of level 0
    DevBuf<int64_t> c_n;       // per subdomain coarse dofs (3 nloc_0)
    DevBuf<int64_t> c_ld;      // per subdomain row stride of its inverse (c_n padded to 4)
    // device node numbering: fine_perm[s][i] = device position (inside member s's segment of
    // the fine level) of the member's node i in the reference (level-ordered) numbering
    std::vector<std::vector<int32_t>> fine_perm;
    // the same for every level: level_perm[l][s][reference local node] = device local node
    std::vector<std::vector<std::vector<int32_t>>> level_perm;
    int64_t fine_dof(int s, int64_t dof) const {  // batch fine-level dof of member s's nodal dof
        return 3 * (lev.back().noff[s] + fine_perm[s][dof / 3]) + dof % 3;
    }
    // condensed <-> nodal map of the fine level, per subdomain (batch-global nodal dofs)
    std::vector<int64_t> nfree;              // per subdomain
    std::vector<std::vector<int32_t>> free_dof_host;
    std::vector<DevBuf<int32_t>> free_dof;

    // PCG work vectors (fine level, 3 nn_L) + per-subdomain scalars
    DevBuf<double> pcg_mem, partial;         // pcg_mem holds the six vectors below
    DevSpan<double> xs, rs, zs, ps, qs, bs;
    DevBuf<double> stage;  // condensed b / x of the C-ABI solve (allocated at create, capi_mgpis.hip)
    DevBuf<PcgScal> sc;
    PcgScal* sc_host = nullptr;      // pinned, filled by pcg_finish()
    MirrorBuf mirror;                // per-subdomain stop state, host-mapped
    DevBuf<int64_t> fin_cb;          // per-subdomain first chunk of the fine level (nsub + 1)

    int64_t fine_dof_offset(int s) const { return 3 * lev.back().noff[s]; }
    int64_t fine_nodes(int s) const { return lev.back().nloc[s]; }

    // ---- operations (all asynchronous on `stream` unless stated)
    // y = K_level x (batch nodal layout); vc_op: the V-cycle's copy of the operator
    void spmv(int level, const double* x, double* y, bool vc_op = false);
    bool vc32() const { return opt.precond_fp32 != 0 && lev.size() > 1; }
    // storage type of the V-cycle's copy of level l (table-mode levels: the table)
    int vc_type(int l) const {
        if (!vc32() || lev[l].tbl) return kVal64;
        return lev[l].val8.p ? kValQ8 : lev[l].val16.p ? kValH16 : kVal32;
    }
    // z = M^-1 r (fine level); dot: leave the partials of r.z (vc_partial)
    void vcycle(const double* r, double* z, bool dot);
    // b_{l-1} = realProl[l-1]^T r_l on every member (masked), batch nodal layouts of levels l, l-1
    void restrict_level(int l, const double* rf, double* bc);
    // block (rotated-node) parts of the transfer from level l-1 to l: b_c += B^T r_f, x_f += B e_c
    void rot_restrict(int l, const double* rf, double* bc, const PcgScal* scp);
    void rot_prolong(int l, const double* ec, double* xf, const PcgScal* scp, float4* xf4 = nullptr);
    // PCG over every subdomain of the batch; b in bs, result in xs (x0 = xs when warm).
    // begin() enqueues the setup, step() one graph replay (iters_per_graph iterations),
    // wait() paces replays on the host-mapped stop flags until every subdomain is done.
    void pcg_begin(int prec, double rtol, const std::vector<int64_t>& maxit, bool warm = false);
    void pcg_step(int prec);
    void pcg_wait(int prec, int64_t pre_enqueued);
    void pcg_fetch();                  // enqueue the copy of the scalars into sc_host
    void pcg_check();                  // after the stream synchronised: timing sample, breakdown
    void pcg_finish();                 // fetch + synchronise + check
    void pcg_solve(int prec, double rtol, const std::vector<int64_t>& maxit, bool warm = false);
    void scatter_free(int s, const double* cond, double* full);   // device pointers
    void gather_free(int s, const double* full, double* cond);
    // timing of the fine-level SpMV (HIP events around it in the eager first iteration)
    hipEvent_t ev_k0 = nullptr, ev_k1 = nullptr;
    double timed_kernel_ms = 0.0;
    double timed_kernel_bytes = 0.0;  // algorithmic bytes of the sampled launches (active members)
    int64_t timed_kernel_samples = 0;
    bool time_kernel = false;
    double fine_kernel_bytes(int s) const;  // algorithmic bytes of the timed kernel, member s
    // Algorithmic HBM bytes of the solve path (every input read once, every output
    // written once, gathered operands counted once per unique element), accumulated by pcg_check
    // over the members' iteration counts: [0] fine-level kernels (the Krylov SpMV, k_axpy and the
    // V-cycle's launches on the fine level, including the transfers to and from it), [1] every
    // launch below the fine level (coarser sweeps, residuals, transfers, the dense coarse solve)
    // and the scalar kernels, [2] launches counted
    double alg_bytes[3] = {0.0, 0.0, 0.0};
    // model per member s: one PCG iteration (SpMV + axpy + V-cycle + scalars), split as above;
    // setup: x0 = 0 initialisation + the first V-cycle
    void iteration_bytes(int s, double out[2]) const;
    void setup_bytes(int s, double out[2]) const;
    void vcycle_bytes(int s, double out[2]) const;
    int64_t iteration_launches() const;
    // operator bytes of one fine pass, member s (prod_cols: with the 16-bit column offsets the
    // production kernels use; the mgpis_gpu_bench_spmv variants read 32-bit columns)
    double fine_matrix_bytes(int s, int vt, bool prod_cols = true) const;
    double bench_spmv(int variant, int reps);  // ms per launch of a fine-level SpMV loop variant
    int64_t graphs_launched = 0;

    // Two-stream split of the batch (set_split before the first solve): the members are dealt
    // into two halves of equal fine work, each half's PCG iterations are a graph of their own
    // replayed on its own stream, so one half's latency-bound coarse levels and kernel
    // boundaries overlap the other half's fine-level streaming.  Each half runs on its own copy
    // of the scalars in which the other half's members are marked done (the kernels already skip
    // done members), so the two graphs touch disjoint chunks; pcg_wait joins the streams and
    // merges the copies back into `sc`.  Setup and the eagerly timed first iteration stay on
    // `stream` over the whole batch.
    // parts > 2 (DDPCA_PCG_STREAMS=n): the same with n parts on n streams (A/B)
    void set_split(bool on, int parts = 2);
    bool split() const { return split_; }
    // capture the PCG graphs of preconditioner prec now (create time) instead of at the first solve
    void prepare_graphs(int prec) { build_graph(prec); }

private:
    hipGraphExec_t graph_[2] = {nullptr, nullptr};
    hipGraphExec_t graph_h_[2][kMaxParts] = {};  // [prec][part]
    // one-iteration graphs for the tail of a solve: once the queued iterations reach the members'
    // expected count (their previous solve's, expect_[prec]), the host queues single iterations
    // two ahead of the slowest member instead of whole replays, so at most two iterations of
    // launches run after the last member converged (a replay of iters_per_graph left up to
    // ~1.5 k over, every launch of it dispatching its full grid to exit at once)
    hipGraphExec_t graph1_[2] = {nullptr, nullptr};
    hipGraphExec_t graph1_h_[2][kMaxParts] = {};
    std::vector<int64_t> expect_[2];
    int last_prec_ = -1;
    int64_t horizon(int prec, int half) const;  // max expected iterations (half -1: all members), INT64_MAX unknown
    bool split_ = false;
    int nparts_ = 1;                          // parts of the split batch (2: the halves)
    hipStream_t xstream_[kMaxParts - 1] = {};  // part h >= 1 replays on xstream_[h - 1], part 0 on `stream`
    hipStream_t part_stream(int h) const { return h == 0 ? stream : xstream_[h - 1]; }
    hipEvent_t ev_fork_ = nullptr, ev_join_[kMaxParts - 1] = {};
    DevBuf<PcgScal> sc_half_;   // nparts_ x nsub: the scalars each part's graph runs on
    DevBuf<int32_t> half_;      // per member: its part
    std::vector<int> half_host_;
    PcgScal* sc_cur_ = nullptr; // the scalars enqueue_iteration / vcycle bind (sc, or a half's copy)
    void build_half_graph(int prec, int h);
    hipGraphExec_t capture_iterations(int prec, int count, PcgScal* scp);
    void launch_fin(hipStream_t st, int what, const double* part, const double* part2, const int64_t* cb, PcgScal* scp,
                    PcgMirror* mir);
    bool sample_pending_ = false;
    bool solve_accounted_ = true;
    void build_graph(int prec);
    void enqueue_iteration(int prec, bool timed);
    void estimate_lmax(int level);
};

// The other drivers of the MGPIS class surface (device_krylov.hip), on member 0 of a one-member
// batch; b, x: device vectors in the fine level's batch nodal layout.  Return iterNumb at exit.
int64_t krylov_mult_solv(MgpisDevice& D, const double* b, double* x, int64_t maxit, double* relres);
// attainable: also stop within 100 rtol once the residual is flat (LAGRANGE only, *breakdown = 2)
int64_t krylov_bicgstab(MgpisDevice& D, int prec, const double* b, double* x, double rtol, int64_t maxit,
                        double* relres, int* breakdown, bool attainable = false);
int64_t krylov_gmres(MgpisDevice& D, int prec, const double* b, double* x, double rtol, int64_t maxit, int64_t restart,
                     double* relres);

}  // namespace ddpca
