/*
 * ddpca_amd.h -- C ABI of libddpca_amd.so, the MI355X-native hot path of DDPCA-ADMM.
 *
 * Drop-in boundary for the per-subdomain solve loop of the reference
 * (QuanchengP/DDPCA-ADMM).  The reference is header-only C++ with no FFI; its interface for
 * this path is the class surface of MGPIS (MGPIS.h:8-38), MULTIGRID (MULTIGRID.h:10-95) and
 * MCONTACT (MCONTACT.h:9-95).  Each entry point below cites the reference member it replaces.
 * Plain pointers and sizes only.  Host pointers are borrowed (copied at create); device memory
 * is owned by the handle.  Return 0 on success, a negative DDPCA_E* code on error; a positive
 * return from a solve is the iteration count when the iteration cap was reached.
 * Handles are independent: calls on different handles may run concurrently from different
 * host threads (the reference calls CG_SOLV concurrently per subdomain, MCONTACT.h:2511), creates
 * included: every graph a handle replays is captured at its create, on the creating thread, under a
 * process-wide capture lock that the library's synchronous allocations and copies also take, so a
 * solve only replays (tests/test_mgpis_gpu.py::test_concurrent_cg_solv_bit_identical).  Calls on
 * ONE handle are not to overlap.
 */
#ifndef DDPCA_AMD_H
#define DDPCA_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DDPCA_OK 0
#define DDPCA_EINVAL (-1)   /* bad argument / shape */
#define DDPCA_EHIP (-2)     /* HIP runtime error */
#define DDPCA_ENOGPU (-3)   /* no gfx950 device visible */
#define DDPCA_ESTATE (-4)   /* call sequence error */
#define DDPCA_ECOMM (-5)    /* RCCL error */
#define DDPCA_ENUMERIC (-6) /* NaN/Inf or breakdown in a Krylov scalar */
#define DDPCA_ENOCONV (-7)  /* iteration cap reached before convergence (LAGRANGE's Newton loop) */

/* last error message of the calling thread (never NULL) */
const char* ddpca_last_error(void);
/* 1 if a gfx950 device is visible, 0 otherwise (no HIP context is created otherwise) */
int ddpca_gpu_available(void);
/* (the measurement probes -- STREAM ceiling, grid barrier -- are in libddpca_probe.so,
 * include/ddpca_probe.h) */

/* ========================================================================================
 * MGPIS -- multigrid-preconditioned CG on one subdomain (MGPIS.h:8-225)
 * ======================================================================================== */
typedef struct ddpca_mgpis* mgpis_t;

typedef struct {
    int smoother;      /* 0 = damped point Jacobi, 1 = 3x3 node-block Jacobi, 2 = Chebyshev(deg) on block Jacobi,
                          3 = multicolour block Gauss-Seidel on the fine level (forward before, backward after
                          the coarse correction; band mode on a refined band) + nu block-Jacobi sweeps below,
                          4 = as 3 with colour SSOR on the fine level (forward + backward before and after,
                          the reference's MULT_VCYC order, MGPIS.h:64-76, 101-114; measured slower, A/B only).
                          4 needs precond_fp32 >= 1 */
    int nu;            /* sweeps (Jacobi) or polynomial degree (Chebyshev) pre and post */
    double omega;      /* Jacobi damping; > 0: this value; 0: 4 / (3 lambda_max(M^-1 K)) estimated at
                          create per level and subdomain; < 0: -omega / lambda_max(M^-1 K)
                          (mgpis_default_options: -1.7, the measured optimum for block Jacobi) */
    int iters_per_graph; /* PCG iterations captured per hipGraph replay (>= 1) */
    int warm_start;    /* MCONTACT loop only: start each subdomain PCG from its previous solution
                          instead of x0 = 0 (MGPIS.h:168); same ||r|| <= rtol ||b|| stop rule */
    int precond_fp32;  /* 1: the V-cycle's level operators are stored rounded to fp32 (once, at
                          create; still exactly symmetric, all arithmetic fp64).  The Krylov
                          operator, vectors and the stop rule stay fp64, so the solution meets the
                          same ||r|| <= rtol ||b||; only the preconditioner differs slightly.
                          2: as 1, and the fine level's V-cycle copy (smoothing sweeps and the
                          V-cycle residual) stored as block-exponent fp16 (2^e x nine fp16 per 3x3
                          block) -- 24 instead of 40 B per block on the two fine smoother passes
                          of every PCG iteration.
                          3: as 2 with block-scaled int8 instead of fp16 (nine int8 and a scale
                          = the block maximum / 127 per 3x3 block) -- 14 B per block.
                          4: as 3, and the V-cycle sweeps gather fp32 stride-4 copies of their
                          iterates (one 16-B load per neighbour): the colour sweeps of smoother
                          3 / 4 on lattice transfers (the fine restriction then reads an fp32 copy
                          of the residual) and every block-Jacobi level with 16-bit columns (only
                          its last sweep writes fp64); products, dot products and the V-cycle
                          output stay fp64. */
    int table_mode;    /* levels >= 1: 0 stream every block value; 1 (default) when the rows'
                          block values deduplicate well (structured meshes), keep one copy per
                          distinct row in a cache-resident table and stream only column indices
                          and a row type -- the operator is bit-identical; 2 force (tests) */
    int coarse_level;  /* level of the exact (dense-inverse) coarse solve of the V-cycle; the reference
                          factorises level 0 (MGPIS.h:58-62).  -1 (default): the highest level whose
                          dense inverses of all batch members fit in 256 MB -- fewer, latency-bound
                          coarse-level launches when a process owns few subdomains */
} mgpis_options_t;

/* Fill default options. */
void mgpis_default_options(mgpis_options_t* opt);

/* Replaces MULTIGRID::CONSTRAINT(1) -> MGPIS::ESTABLISH() (MULTIGRID.h:1245-1252,
 * MGPIS.h:40-53): uploads the level hierarchy in the reference's own layout.
 *   nlev                       = maxiLeve + 1
 *   nnodes[l]                  nodes of level <= l (level-ordered numbering, MULTIGRID.h:884-910)
 *   nfree[l]                   rows of consStif[l]
 *   free_dof[l][i]             nodal dof (3*node + comp) of condensed row i (consOper[l])
 *   K_ptr/K_col/K_val[l]       consStif[l] as CSR (int64 row pointer, int32 columns)
 *   S_ptr/S_col/S_w[l]         scalar stencil scalProl[l], nnodes[l+1] x nnodes[l], l < nlev-1
 *                              (realProl[l] = consOper[l+1] (S (x) I3) consOper[l]^T)
 * The coarse level is inverted once here (the reference re-factorises it on every CG_SOLV
 * call, MGPIS.h:185). */
int mgpis_gpu_create(int device, int nlev, const int64_t* nnodes, const int64_t* nfree,
                     const int32_t* const* free_dof, const int64_t* const* K_ptr,
                     const int32_t* const* K_col, const double* const* K_val,
                     const int64_t* const* S_ptr, const int32_t* const* S_col,
                     const double* const* S_w, const mgpis_options_t* opt, mgpis_t* out);

/* Same as mgpis_gpu_create, with the transfers given as the reference's own
 * MGPIS::realProl[l] (condensed CSR, nfree[l+1] x nfree[l], MULTIGRID.h:1141-1181, 1246-1249)
 * instead of the scalar stencil, so hierarchies with rotated nodes (MULTIGRID::nodeRota: CYLINDER,
 * DEHW hubs) drop in unchanged: every (fine node, coarse node) block whose free part is w*I runs as
 * a stencil weight, every other 3x3 block as a block entry (k_prolong_rot / k_restrict_rot).
 * DDPCA_EINVAL when a coarse node's row is not the identity. */
int mgpis_gpu_create_prol(int device, int nlev, const int64_t* nnodes, const int64_t* nfree,
                          const int32_t* const* free_dof, const int64_t* const* K_ptr,
                          const int32_t* const* K_col, const double* const* K_val,
                          const int64_t* const* P_ptr, const int32_t* const* P_col,
                          const double* const* P_val, const mgpis_options_t* opt, mgpis_t* out);

/* Same hierarchy in node-block form: B_*[l] is the UNCONSTRAINED Galerkin operator
 * origStif[l] (MULTIGRID.h:1182-1184) as 3x3-block CSR (9 doubles per block, row-major);
 * dof_free[3*nnodes[nlev-1]] marks free dofs (consFlag, MULTIGRID.h:1186-1194). */
int mgpis_gpu_create_bsr3(int device, int nlev, const int64_t* nnodes,
                          const int64_t* const* B_ptr, const int32_t* const* B_col,
                          const double* const* B_val, const uint8_t* dof_free,
                          const int64_t* const* S_ptr, const int32_t* const* S_col,
                          const double* const* S_w, const mgpis_options_t* opt, mgpis_t* out);

/* Replaces MGPIS::CG_SOLV(precSwit, totaForc, resuSolu) (MGPIS.h:163-225):
 * x0 = 0, stop when ||r|| <= rtol * ||b|| on the recursive residual (reference rtol = 1e-14)
 * or after maxit iterations (reference maxit = rows).  prec: 0 diagonal (DIAG_PREC,
 * PREP.h:393-401), 1 multigrid V-cycle.  b, x are condensed host vectors of length nfree[L].
 * iters/relres may be NULL.  Returns 0, or maxit (> 0) when the cap was hit. */
int mgpis_gpu_solve(mgpis_t h, const double* b, double* x, int prec, double rtol,
                    int64_t maxit, int64_t* iters, double* relres);

/* Replaces MGPIS::MULT_SOLV(totaForc, resuSolu) (MGPIS.h:130-160): x0 = 0, repeated V-cycles
 * x <- MULT_VCYC(b, x) until the last five residual norms ||b - Kx|| oscillate by less than 0.1
 * of their median (VECT_MEDI_OSCI, PREP.h:147-153), or maxit V-cycles (reference 10000).
 * iters = the reference's iterNumb at exit (the value it prints); relres = ||b - Kx|| / ||b||.
 * The cycle is the handle's (options): a stagnation rule returns the accuracy the cycle's
 * contraction allows -- use nu >= 2 (block-Jacobi V(2,2) matches SGS V(1,1), tests).
 * Returns 0, or maxit (> 0) when the cap was hit. */
int mgpis_gpu_mult_solve(mgpis_t h, const double* b, double* x, int64_t maxit, int64_t* iters, double* relres);
/* Replaces MGPIS::BiCGSTAB_SOLV(precSwit, totaForc, resuSolu) (MGPIS.h:350-432): right-
 * preconditioned BiCGSTAB, x0 = 0, shadow residual b, stop on the recursive residual
 * ||r|| <= rtol ||b|| (reference 1e-14) or maxit (reference = rows).  *breakdown (may be NULL)
 * = 1 when rho = 0 ended the run (the reference's "ERROR 1" exit, MGPIS.h:386-389) -- like the
 * reference, x is then returned as it stands.  These are the only stop rules of this entry point
 * (LAGRANGE's Newton steps add an attainable-accuracy stop, see ddpca_lagrange_get).  Returns 0,
 * maxit on the cap, DDPCA_ENUMERIC on NaN/Inf. */
int mgpis_gpu_bicgstab(mgpis_t h, const double* b, double* x, int prec, double rtol, int64_t maxit,
                       int64_t* iters, double* relres, int* breakdown);
/* Replaces MGPIS::GMRES_SOLV(precSwit, totaForc, resuSolu) (MGPIS.h:228-348): left-preconditioned
 * GMRES(restart) (reference restart = iterStag = 10, rtol = 1e-12, maxit = rows), classical
 * Gram-Schmidt Arnoldi; stop on the true residual: <= rtol ||b||, or <= 100 rtol ||b|| with the
 * last `restart` residuals oscillating by less than 0.1 of their median.  restart in [1, 24].
 * iters = iterNumb at exit; relres = ||b - Kx|| / ||b||.  Returns 0, or maxit on the cap. */
int mgpis_gpu_gmres(mgpis_t h, const double* b, double* x, int prec, double rtol, int64_t maxit,
                    int64_t restart, int64_t* iters, double* relres);
/* y = consStif[level] * x (condensed host vectors), for parity tests of the SpMV kernel. */
int mgpis_gpu_spmv(mgpis_t h, int level, const double* x, double* y);
/* The same through the V-cycle's stored copy of the fine level (vcycle_copy = 1: fp32,
 * block-exponent fp16 or block-scaled int8 values per precond_fp32; DDPCA_EINVAL without one),
 * or the fp64 operator (0) -- the decode of the reduced-precision records against their host
 * rounding, for parity tests. */
int mgpis_gpu_spmv_copy(mgpis_t h, int level, int vcycle_copy, const double* x, double* y);
/* z = M^-1 r: one V-cycle from zero (MGPIS::MULT_VCYC, MGPIS.h:55-128) on condensed vectors. */
int mgpis_gpu_vcycle(mgpis_t h, const double* r, double* z);
/* Informational: [nlev, n_fine_free, nnzb_fine, chunks_fine, omega*1e6, lambda_max*1e6, device] */
int mgpis_gpu_info(mgpis_t h, int64_t* out7);
/* Diagnostic (no reference counterpart): average ms per launch of a fine-level SELL-BSR3
 * kernel over `reps` back-to-back launches on this operator.  variant = loop (0 cached x3
 * unroll, 1 non-temporal matrix loads, 2 column prefetch + non-temporal, 3 a bound only: x
 * gathered at the row's own node, wrong values) + 4 * mode (0 y = Kx, 1 PCG q = Kz + beta q,
 * p = z + beta p with p.q, 2 residual b - Kx, 3 Chebyshev sweep on block Jacobi).
 * bytes (may be NULL) = algorithmic bytes per launch. */
int mgpis_gpu_bench_spmv(mgpis_t h, int variant, int reps, double* ms, double* bytes);
int mgpis_gpu_destroy(mgpis_t h);

/* ========================================================================================
 * Host problem construction (setup only, not on the hot path): the reference's MULTIGRID
 * mesh/operator pipeline and MCONTACT::ESTABLISH restated in C++ (mcontact.cpp,
 * multigrid.cpp).  Produces the operands of the device path.
 * ======================================================================================== */
typedef struct ddpca_problem* ddpca_problem_t;

/* kind / params:
 *   "beam"     d0 d1 d2 globLeve D0 D1 D2       BEAM.h (D = 1,1,1: MESH_NODD; else MESH_DD,
 *                                              glued interfaces fricCoef = -1, BEAM.h:424-470)
 *   "twoblock" fric globLeve                    two stacked blocks, one contact interface
 *   "dehw"     ngroups nx ny nz globLeve fric [kc kg]
 *                                              synthetic DEHW-shaped chain: per group one
 *                                              worm and one wheel block in frictional contact,
 *                                              groups glued along x (worm-worm, wheel-wheel);
 *                                              kc / kg (default 0): contact / glued faces
 *                                              integrated over 2^k x 2^k polygons each (the
 *                                              intersection with a 2^k times finer slave mesh) */
int ddpca_problem_create(const char* kind, const double* params, int nparams, ddpca_problem_t* out);
/* Replace the integration points of interface ts (CSEARCH::intePoin, CSEARCH.h:19-32):
 * node[n][2][4], shap[n][2][4], basis[n][3][3], gap[n], w[n]. */
int ddpca_problem_set_ips(ddpca_problem_t p, int64_t ts, int64_t n, const int64_t* node,
                          const double* shap, const double* basis, const double* gap,
                          const double* w, double fric, double penN, double penF);
/* CSEARCH::BUCKET_SORT + CONTACT_SEARCH (CSEARCH.h:205-230, 777-817; per face pair
 * SEGMENT_INTERSECT / SI_SUB 614-775): the integration points of the contact between a master and
 * a slave face set, in the reference's order.
 *   mast_xyz[3 * mast_nnode], slav_xyz[3 * slav_nnode]  node coordinates by node id
 *   mast_segm[4 nm], slav_segm[4 ns]                     4 node ids per face (EFACE_SURFACE order)
 *   mast_2d[2 nm], slav_2d[2 ns]                         the faces' 2-D bucket coordinates (the
 *                                                        examples' mastCoor / slavCoor)
 *   buck[2]                                              bucket counts (buckNumb)
 *   maxiDist                                             keep a face pair when one of its points has
 *                                                        initial gap <= maxiDist (reference 1e12)
 * The result feeds ddpca_problem_set_ips (ddpca_ips_get's layout is set_ips'). */
typedef struct ddpca_ips* ddpca_ips_t;
int ddpca_contact_search(const double* mast_xyz, int64_t mast_nnode, const double* slav_xyz, int64_t slav_nnode,
                         int64_t nm, const int64_t* mast_segm, const double* mast_2d, int64_t ns,
                         const int64_t* slav_segm, const double* slav_2d, const int64_t* buck, double maxiDist,
                         ddpca_ips_t* out);
/* CSEARCH::ADAPTIVE_REFINE (CSEARCH.h:839-956), the selection: with the same face / bucket input as
 * ddpca_contact_search, every node of the integration points of face pairs that come within
 * distCrit is a split node, and a candidate element (8 corner node ids; the caller passes the leaf
 * elements of level tempLeve) with a split corner is flagged in mast_split / slav_split.  Returns
 * 1 when any node was selected (the reference's isnoRefi), 0 otherwise.  Refining the flagged
 * elements (CURVEDS::REFINE + MULTIGRID::REFINE, refiPatt 0) is the caller's mesh operation. */
int ddpca_refine_select(const double* mast_xyz, int64_t mast_nnode, const double* slav_xyz, int64_t slav_nnode,
                        int64_t nm, const int64_t* mast_segm, const double* mast_2d, int64_t ns,
                        const int64_t* slav_segm, const double* slav_2d, const int64_t* buck, double distCrit,
                        int64_t ne_m, const int64_t* mast_elem, int64_t ne_s, const int64_t* slav_elem,
                        uint8_t* mast_split, uint8_t* slav_split);
int64_t ddpca_ips_count(ddpca_ips_t h);
/* node[n][2][4], shap[n][2][4], basis[n][3][3] (n, t1, t2), gap[n], w[n]; any pointer may be NULL */
int ddpca_ips_get(ddpca_ips_t h, int64_t* node, double* shap, double* basis, double* gap, double* w);
int ddpca_ips_destroy(ddpca_ips_t h);
/* Coarse-space setting of MCONTACT (muscSett / doleMcsc, MCONTACT.h:22-23), before establish.
 * muscSett = 2 selects the interface-eliminated coarse space (MULTISCALE_1, MCONTACT.h:
 * 1672-2301; the examples' choice, e.g. BLOCK.h:38, TORSION.h:39, DEHW.h:2222), built by
 * establish and applied by every ADMM iteration while tc <= MULT_MAXI (MCONTACT.h:2578-2612);
 * doleMcsc[tv] = coarse level of subdomain tv (NULL = 0).  muscSett = 0 (default): none.
 * muscSett = 1 selects the LATIN-type space (MULTISCALE, MCONTACT.h:898-1536, CYLINDER.h:42;
 * applied as MCONTACT.h:2540-2576), assembled by establish (rank-locally under
 * ddpca_problem_establish_owned: each rank its own rows and interface sides, summed on the device
 * by RCCL).  3 (both) is DDPCA_EINVAL. */
int ddpca_problem_set_coarse(ddpca_problem_t p, int64_t muscSett, const int64_t* doleMcsc);
/* MCONTACT::ESTABLISH (MCONTACT.h:181-896); single grids just run TRANSFER / STIF_MATR /
 * CONSTRAINT(1). */
int ddpca_problem_establish(ddpca_problem_t p);
/* Rank-local ESTABLISH: operators only for subdomains with owner[tv] == rank and for the
 * interfaces touching them (each process of a multi-GPU run builds its own share). */
int ddpca_problem_establish_owned(ddpca_problem_t p, const int32_t* owner, int rank);
/* Read-only view of an internal array.  dtype: 0 float64, 1 int64, 2 int32, 3 uint8.
 * Names: see ddpca_amd.py (_ARRAYS). index = subdomain, level or 2*interface+side. */
int ddpca_problem_view(ddpca_problem_t p, const char* name, int64_t index, int64_t level,
                       const void** data, int64_t* count, int* dtype);
int ddpca_problem_destroy(ddpca_problem_t p);
/* Build the device solver of subdomain tv from the problem (mgpis_gpu_create_bsr3). */
int ddpca_problem_mgpis(ddpca_problem_t p, int64_t tv, int device, const mgpis_options_t* opt,
                        mgpis_t* out);

/* ---- Operator-level builder: a caller that already holds the reference's operators (its
 * MULTIGRID/MGPIS hierarchy per subdomain and the interface operators of MCONTACT::ESTABLISH,
 * MCONTACT.h:181-896) hands them over in the reference's layouts; after finalize the problem
 * is established and mcontact_gpu_create / ddpca_problem_mgpis accept it.  The host
 * restatement is bypassed. */
typedef struct {
    int64_t nrow, ncol;
    const int64_t* ptr;  /* nrow + 1 */
    const int32_t* col;
    const double* val;
} ddpca_csr_t;

int ddpca_problem_empty(int64_t nsub, int64_t nint, ddpca_problem_t* out);
/* Subdomain tv: the MGPIS hierarchy exactly as mgpis_gpu_create takes it (nnodes, nfree,
 * free_dof, consStif[l] CSR, scalar stencils scalProl[l]), consForc (nfree[nlev-1] condensed
 * load, MULTIGRID::consForc), presc (3*nnodes[nlev-1] nodal values, read at constrained dofs:
 * the Dirichlet values OUTP_SUB1 writes, MULTIGRID.h:1263-1281; NULL = 0) and coords
 * (3*nnodes[nlev-1] node coordinates, level-ordered; NULL = keep the reference node order on
 * the device). */
int ddpca_problem_set_subdomain(ddpca_problem_t p, int64_t tv, int nlev, const int64_t* nnodes,
                                const int64_t* nfree, const int32_t* const* free_dof,
                                const int64_t* const* K_ptr, const int32_t* const* K_col,
                                const double* const* K_val, const int64_t* const* S_ptr,
                                const int32_t* const* S_col, const double* const* S_w,
                                const double* consForc, const double* presc, const double* coords);
/* Same, with the transfers as the reference's MGPIS::realProl[l] (condensed CSR, nfree[l+1] x
 * nfree[l], MULTIGRID.h:1141-1181, 1246-1249) instead of scalProl -- hierarchies with rotated nodes
 * (MULTIGRID::nodeRota: DEHW hubs) whose w R_off^T R_par blocks a scalar stencil cannot hold; the
 * blocks run as block entries (as mgpis_gpu_create_prol). */
int ddpca_problem_set_subdomain_prol(ddpca_problem_t p, int64_t tv, int nlev, const int64_t* nnodes,
                                     const int64_t* nfree, const int32_t* const* free_dof,
                                     const int64_t* const* K_ptr, const int32_t* const* K_col,
                                     const double* const* K_val, const int64_t* const* P_ptr,
                                     const int32_t* const* P_col, const double* const* P_val,
                                     const double* consForc, const double* presc, const double* coords);
/* The hanging level of subdomain tv (after set_subdomain, before its interfaces): locally refined
 * meshes (CYLINDER) put hanging nodes -- and coupled nodes -- on a level maxiLeve + 1 outside the
 * MGPIS hierarchy (MULTIGRID.h:836-848, 884-910); OUTP_SUB1 gives them prolOper[maxiLeve] of the
 * level-maxiLeve vector (MULTIGRID.h:1279).  nnodes_all = all nodes of the subdomain (the
 * interface operators' 3 N columns / rows); hang = rows 3 nnodes[nlev-1] .. 3 nnodes_all - 1 of
 * prolOper[maxiLeve] in the position numbering (3 (nnodes_all - nnodes[nlev-1]) x
 * 3 nnodes[nlev-1]).  The device keeps those values in u as well: MONITOR's norms, resuDisp and the
 * interface products see every node, and the body-balance RHS folds the hanging rows in
 * (ADDITIONAL_FORCE's prolOper^T, MULTIGRID.h:1257-1261). */
int ddpca_problem_set_hanging(ddpca_problem_t p, int64_t tv, int64_t nnodes_all, const ddpca_csr_t* hang);

/* ---- the MULTIGRID operator pipeline on a caller's element tree (host only, capi_multigrid.cpp)
 * Replaces MULTIGRID::TRANSFER + PATCH + STIF_MATR + CONSTRAINT(1) (MULTIGRID.h:722-1255) for any
 * octree the reference's REFINE / GRLE_CHECK produced: every refinement pattern, local refinement
 * (hanging nodes on the level maxiLeve + 1, moved to their parents' average by PATCH), coupled
 * nodes (coupNode / coupReps), nodal rotations (nodeRota).
 *   create: nnode node ids 0..nnode-1 with coordinates (3 per node: nodeCoor); per element e
 *     (elemVect order): corner[8e..8e+7] (cornNode), parent[e] (-1 at level 0), level[e],
 *     refiPatt[e] (the pattern a refined element was split with, 0..6; 7 = leaf), children
 *     child[child_ptr[e] .. child_ptr[e+1]) (TREE_ELEM::children, empty = leaf).
 *   set: "consDofv" (n node-id dofs 3 node + comp, val = prescribed value; set BEFORE the loads,
 *     as the reference requires), "exteForc" (n dofs, val: LOAD_ACCU in order; loads on
 *     constrained dofs are dropped), "nodeRota" (n nodes, val = 9 n, row-major 3x3 each),
 *     "coupNode" (n nodes), "coupReps" (n = 1: the representative node or -1), "material"
 *     (n = 2: val = {mateElas, matePois}; default 210e9, 0.3).
 *   build: TRANSFER, PATCH, STIF_MATR, origStif += extra (nullable: 3 nnode x 3 nnode CSR in
 *     node ids, e.g. the contact interfaces' systMass, MCONTACT.h:816-822), CONSTRAINT(1).
 *   view (after build; same dtype codes as ddpca_problem_view): "posiNode" (int64 per position:
 *     the node id, i.e. earlTran), "nodeCoor" (3 per node id, after PATCH), "leveCount" (int64,
 *     cumulative positions per level 0..maxiLeve, then the total incl. the hanging level),
 *     "freeCount", "consFlag" (uint8 per position dof), "consForc", "dispForc", and CSR parts
 *     ("<X>:ptr|col|val|shape") of "K" (MGPIS::consStif[level]), "P" (MGPIS::realProl[level],
 *     level+1 <- level) and "H" (rows 3 NL.. of prolOper[maxiLeve], positions: the hanging level).
 *   set_subdomain_multigrid: subdomain tv of an operator-level problem from the built tree (what
 *     set_subdomain(_prol) + set_hanging take from the reference's own MULTIGRID); interface
 *     operators handed over afterwards are in the position numbering (posiNode maps them). */
typedef struct ddpca_multigrid* ddpca_multigrid_t;
int ddpca_multigrid_create(int64_t nnode, const double* coords, int64_t nelem, const int64_t* corner,
                           const int64_t* parent, const int64_t* level, const int64_t* refiPatt,
                           const int64_t* child_ptr, const int64_t* child, ddpca_multigrid_t* out);
int ddpca_multigrid_set(ddpca_multigrid_t g, const char* what, int64_t n, const int64_t* idx, const double* val);
/* refine (before build): MULTIGRID::REFINE (MULTIGRID.h:375-545) -- GRLE_CHECK's level balancing
 * (the leaf neighbours across the refined elements' parent edges / faces join with pattern 0),
 * then the n leaf elements elem[] are cut with patterns patt[] (0 xi-eta-zeta 8-way, 1 xi-eta,
 * 2 eta-zeta, 3 zeta-xi 4-way, 4 xi, 5 eta, 6 zeta 2-way).  A new node takes planSurf's position
 * when its corner set is a key there (nplan keys: plan_node[plan_ptr[q] .. plan_ptr[q+1]), position
 * plan_xyz[3q..3q+2]: the caller's curved surface, CURVEDS::REFINE's output), else the corners'
 * average; nodes are deduplicated by coordinates as TRY_ADD_NODE does (1e-10).  spliFlag (nflag
 * pairs: element, child index) selects children for the next round: ddpca_multigrid_tree
 * "nextSplit". */
int ddpca_multigrid_refine(ddpca_multigrid_t g, int64_t n, const int64_t* elem, const int64_t* patt, int64_t nplan,
                           const int64_t* plan_ptr, const int64_t* plan_node, const double* plan_xyz, int64_t nflag,
                           const int64_t* flag_elem, const int64_t* flag_child);
/* CURVEDS (CURVEDS.h:8-121): a curved surface as an ni x nj grid of points (xyz row-major,
 * present[i nj + j] = 0 for grid cells the reference leaves empty; NULL = all present).
 * ddpca_curveds_plan = CURVEDS::REFINE (CURVEDS.h:58-101): for every line and face of the n
 * elements of the (unbuilt) multigrid g whose corners are all grid points, the new node's position
 * = the point at the corners' averaged indices -- the planSurf of ddpca_multigrid_refine (keys as
 * CSR of sorted node ids); the arrays stay valid until the next plan call on c.  Several surfaces:
 * concatenate their plans in the order the reference calls their REFINE (the first entry of a key
 * wins, as planSurf.insert).  ddpca_curveds_rigid = RIGI_ROTR (p <- R p + t, R row-major). */
typedef struct ddpca_curveds* ddpca_curveds_t;
int ddpca_curveds_create(int64_t ni, int64_t nj, const double* xyz, const uint8_t* present, ddpca_curveds_t* out);
int ddpca_curveds_rigid(ddpca_curveds_t c, const double* R, const double* t);
int ddpca_curveds_plan(ddpca_curveds_t c, ddpca_multigrid_t g, int64_t n, const int64_t* elem, const int64_t** plan_ptr,
                       const int64_t** plan_node, const double** plan_xyz, int64_t* nplan);
int ddpca_curveds_destroy(ddpca_curveds_t c);
/* The tree before build (int64 unless noted): "nodeCoor" (f64, 3 per node), "corner" (8 per element),
 * "parent", "level", "refiPatt", "child_ptr" (elements + 1), "child", "nextSplit". */
int ddpca_multigrid_tree(ddpca_multigrid_t g, const char* what, const void** data, int64_t* count, int* dtype);
int ddpca_multigrid_build(ddpca_multigrid_t g, const ddpca_csr_t* extra);
int ddpca_multigrid_view(ddpca_multigrid_t g, const char* what, int64_t level, const void** data, int64_t* count,
                         int* dtype);
int ddpca_problem_set_subdomain_multigrid(ddpca_problem_t p, int64_t tv, ddpca_multigrid_t g);
/* The whole MCONTACT::ESTABLISH (MCONTACT.h:181-896) from element trees: subdomain tv of an empty
 * problem (ddpca_problem_empty) takes a copy of the UNBUILT multigrid g (its tree and the inputs
 * set with ddpca_multigrid_set: constraints, loads, rotations, coupled nodes, material);
 * ddpca_problem_set_contact gives interface ts its bodies (contBody) and ddpca_problem_set_ips its
 * integration points in node ids; ddpca_problem_set_coarse, then ddpca_problem_establish run the
 * library's own pipeline: TRANSFER + PATCH (positions), the mortar operators with CONT_ROTA, STIF_MATR
 * + systMass, CONSTRAINT(1), and MULTISCALE / MULTISCALE_1 on these general trees (the hanging level,
 * prolOper's rotation blocks).  Afterwards the problem's arrays are in the position numbering. */
int ddpca_problem_set_subdomain_tree(ddpca_problem_t p, int64_t tv, ddpca_multigrid_t g);
int ddpca_problem_set_contact(ddpca_problem_t p, int64_t ts, int64_t body0, int64_t body1);
int ddpca_multigrid_destroy(ddpca_multigrid_t g);
/* Interface ts between contBody {body0, body1} with fricCoef fric (< 0 glued, 0 frictionless,
 * > 0 Coulomb; comp = 1 if fric == 0 else 3), nip integration points, nnc_s contact nodes per
 * side; pemaDiag / inpoNgap have comp*nip entries.  ops[7*s + k] is side s's
 *   k = 0 inpoLagr (comp*nip x comp*nnc_s)     1 pemaInpo_r (comp*nip x 3N_s)
 *       2 systTran (3N_s x comp*nnc_s)         3 systTran_pena (3N_s x comp*nnc_s)
 *       4 inteMass (comp*nnc_s square)          5 inteMass_pena (comp*nnc_s square)
 *       6 inteInpo (comp*nnc_s x comp*nip)
 * (MCONTACT.h:213-810).  Set both subdomains first. */
int ddpca_problem_set_interface(ddpca_problem_t p, int64_t ts, int64_t body0, int64_t body1, double fric,
                                int64_t nip, int64_t nnc0, int64_t nnc1, const double* pemaDiag,
                                const double* inpoNgap, const ddpca_csr_t* ops);
/* The caller's own interface-eliminated coarse space (MCONTACT::MULTISCALE_1, MCONTACT.h:
 * 1672-2301, muscSett = 2), after every subdomain and interface was set: doleMcsc[nsub],
 * baseReco[nsub+1], globCoup_1 (n x n), globForc_1 (n), globTran_1[2*ts+s] (n x comp*nnc_s),
 * globTran_D_1[tv] (n x 3N_tv, columns in the nodal numbering of set_subdomain) and
 * accuProl[tv] (nfree_L x nfree_doleMcsc) -- the ADMM loop then applies the correction of
 * MCONTACT.h:2578-2612 every iteration while tc <= MULT_MAXI. */
int ddpca_problem_set_coarse_operators(ddpca_problem_t p, int64_t muscSett, const int64_t* doleMcsc,
                                       const int64_t* baseReco, const ddpca_csr_t* globCoup_1,
                                       const double* globForc_1, const ddpca_csr_t* globTran_1,
                                       const ddpca_csr_t* globTran_D_1, const ddpca_csr_t* accuProl);
/* The caller's own LATIN-type coarse space (MCONTACT::MULTISCALE, MCONTACT.h:898-1536,
 * muscSett = 1, CYLINDER.h:42): doleMcsc[nsub], baseReco[nsub+1], globCoup (n x n: the
 * displacement blocks plus the coarse contact unknowns, rows >= baseReco[nsub]),
 * globTran / globTran_pena [2*ts+s] (n x comp*nnc_s), globTran_D[2*ts+s] (n x 3N of body s,
 * columns in set_subdomain's nodal numbering), accuProl[tv].  Each ADMM iteration then adds
 * u += OUTP_SUB1(accuProl globCoup^-1 sum(globTran l - globTran_pena aux + globTran_D u))
 * (MCONTACT.h:2540-2576) while tc <= MULT_MAXI; globCoup is factorised by pivoted LU. */
int ddpca_problem_set_coarse_latin(ddpca_problem_t p, const int64_t* doleMcsc, const int64_t* baseReco,
                                   const ddpca_csr_t* globCoup, const ddpca_csr_t* globTran,
                                   const ddpca_csr_t* globTran_pena, const ddpca_csr_t* globTran_D,
                                   const ddpca_csr_t* accuProl);
/* The coarse contact unknowns of interface ts of a LATIN coarse space (MULTISCALE's local coarNode,
 * MCONTACT.h:903-957: the level-doleMcsc positions of contBody[ts][0] whose scalEarl * scalProl
 * chain reaches a contact node, increasing), after ddpca_problem_set_coarse_latin.  Optional:
 * with them a coarse problem of DIRE_MAXI = 120000 rows or more is solved by DOUBLE_M's MGPIS
 * (MCONTACT.h:1538-1670, 2558-2559) as the reference does; without them only the dense solve. */
int ddpca_problem_set_coarse_nodes(ddpca_problem_t p, int64_t ts, int64_t n, const int64_t* nodes);
/* Check that every subdomain and interface was set; mark the problem established. */
int ddpca_problem_finalize(ddpca_problem_t p);

/* ========================================================================================
 * MCONTACT -- the ADMM loop of CONTACT_ANALYSIS on the GPU (MCONTACT.h:2493-2845)
 * One handle per process (= per GPU); it owns the subdomains assigned to its rank (solved as
 * one batch) and the interface sides that belong to them.  Interfaces whose sides live on
 * different ranks swap their gamma halves with one grouped RCCL send/recv pair per iteration;
 * the MONITOR norms take one small RCCL all-reduce.
 * ======================================================================================== */
typedef struct ddpca_mcontact* mcontact_t;

/* owner[tv] = rank owning subdomain tv (all ranks pass the same array). */
int mcontact_gpu_create(ddpca_problem_t p, int device, int rank, int nranks,
                        const int32_t* owner, const mgpis_options_t* opt, mcontact_t* out);
/* RCCL communicator from an ncclUniqueId (128 bytes) produced by rank 0 and broadcast by the
 * caller (e.g. through torch.distributed); required when nranks > 1.  With nranks == 1 it is
 * optional: the per-iteration all-reduces (MONITOR norms, coarse right-hand side) then run through
 * a one-rank RCCL communicator, bit-identical to the run without one. */
int mcontact_gpu_comm_init(mcontact_t h, const void* nccl_unique_id);
/* Transport check (no reference counterpart): every rank sends two tagged messages of n doubles to
 * every rank (itself included) in one grouped exchange -- the path the gamma halves take
 * (MCONTACT.h:2632-2636 shares them in memory) -- and all-reduces n doubles (the MONITOR / coarse
 * right-hand-side path); DDPCA_ECOMM unless every element arrives exact.  Collective: all ranks call
 * it (in-process ranks from their own threads). */
int mcontact_gpu_comm_check(mcontact_t h, int64_t n);
/* 128-byte ncclUniqueId for rank 0 to broadcast. */
int mcontact_gpu_unique_id(void* out128);
/* Test transport (no reference counterpart): connects the n handles of ONE process, handles[r] =
 * rank r of n, through host-staged copies instead of RCCL -- the same exchanges (gamma halves of
 * cross-rank interfaces, MONITOR and coarse-RHS all-reduces, the setup all-reduce of the coarse
 * matrix) with the same multi-rank bookkeeping, so a multi-rank run can be checked on one GPU.
 * Each handle's mcontact_gpu_iterate must then be called from its own host thread. */
int mcontact_gpu_comm_local(mcontact_t* handles, int n);
/* Timing transport (no reference counterpart; profiles/one_rank_probe.py): one rank of an
 * nranks > 1 layout alone on a GPU.  Every receive from peer p gets what this rank sent p (an
 * on-device copy on the solve stream) and the all-reduces keep this rank's own values, so the
 * numbers are NOT the N-rank answer but the work is one rank's: its subdomains' solves, its
 * interface sides, its rows of the coarse solve, with the communication left out.  p = the
 * problem h was created from, established in full: it completes the dense coarse operator that the
 * setup all-reduce would sum. */
int mcontact_gpu_comm_loopback(mcontact_t h, ddpca_problem_t p);
/* Run up to maxit ADMM iterations (reference maxiIter = 3000) from the current state;
 * stop on MONITOR convergence (MCONTACT.h:2725-2845) when check != 0.
 * Returns the number of iterations run (>= 0) or a negative error. */
int64_t mcontact_gpu_iterate(mcontact_t h, int64_t maxit, int check);
/* Number of resuMoni columns (2*nsub + 8*nint + 2) and the monitor rows recorded so far
 * (row-major, rows x cols) -- same columns as resuMoni.txt. */
int64_t mcontact_gpu_monitor(mcontact_t h, double* out, int64_t cap_rows);
/* Copy state to host: what = "resuDisp" (index = subdomain, nodal 3N), "inteAuxi"/"inteLagr"
 * (index = 2*ts+side), "inpoGamm" (index = ts, projected gamma of the last iteration),
 * "fricStat" (index = ts, int32 per integration point: 0 open, 1 slip, 2 stick, MCONTACT.h:2647-2666),
 * "pcg_iters" (int64 per owned subdomain, last iteration), "mass_iters" (int64: surface-mass CG
 * iterations of the last iterate call), "coarse_solve" (int64 x4: coarse rows, DOUBLE_M?, dense
 * bytes, dense fallback?), "gs_rows" (int64 x3: the fine rows the multicolour sweeps cover, the
 * band mode's ring and far rows -- 0, 0 without it), "gs_launch_bytes" (the sweeps' per-launch byte
 * model, doubles). */
int64_t mcontact_gpu_get(mcontact_t h, const char* what, int64_t index, void* out, int64_t cap);
/* Timing of the last iterate() call, summed over its iterations: [total_ms (host wall),
 * solve_ms (host wall of the body balance), iface_ms (device, interface step + monitor),
 * comm_ms (device, gamma exchange), spmv_kernel_ms (device events around sampled fine-level
 * SpMV launches), spmv_samples, pcg_iterations (summed over owned subdomain solves),
 * spmv_bytes_per_launch (algorithmic), dof_iterations (sum n_free * PCG its), owned_dofs] */
int mcontact_gpu_timing(mcontact_t h, double* out10);
/* Algorithmic HBM bytes of the last iterate() call, summed over its iterations (SURVEY §8 d4:
 * streamed operators and every vector read / written once, gathered operands once per distinct
 * element; each kernel's model in DESIGN.md §3).  out[0] fine-level PCG kernels (Krylov SpMV,
 * k_axpy, the V-cycle's fine-level sweeps, residuals and transfers), [1] V-cycle launches below
 * the fine level + the PCG scalar kernels, [2] coarse-space correction, [3] body-balance RHS and
 * OUTP_SUB1, [4] interface products + projection, [5] batched surface-mass CG, [6] MONITOR
 * snapshots and norms, [7] body-balance PCG kernel launches (not bytes).  Returns the count (8);
 * copies min(8, cap) when out != NULL.  No equivalent in the reference (measurement only). */
int64_t mcontact_gpu_bytes(mcontact_t h, double* out, int64_t cap);
int mcontact_gpu_destroy(mcontact_t h);
/* The batched surface-mass solver of the ADMM loop on its own (replaces the interface mass solves
 * of MCONTACT.h:2671-2704: SimplicialLDLT below 120000 rows, MCONTACT.h:838-847, Eigen CG above,
 * 2680-2682): nsys square CSR systems A[s], right-hand sides b and solutions x concatenated in
 * system order; Jacobi-PCG per system from x0 = 0 to ||r|| <= rtol ||b|| or maxit -- by default
 * started by a fixed-length Chebyshev iteration on D^-1 A (bounds from 60 Lanczos steps and
 * Gershgorin at setup; skipped for the batch when a bound is not positive or the steps exceed 120;
 * DDPCA_MASS_CHEB=0 turns it off), the CG then restarting from its iterate, iters[] counting the
 * CG's iterations after the restart.  fuse_alpha:
 * -1 the production rule (alpha inside the update kernel up to 1024 chunks per system), 0 / 1
 * force the separate / fused alpha launch.  iters[nsys] (may be NULL).  On a breakdown (p.q <= 0
 * or not finite) the system's x is its last good iterate and the call returns DDPCA_ENUMERIC. */
int ddpca_mass_solve(int device, int64_t nsys, const ddpca_csr_t* A, const double* b, double* x, double rtol,
                     int64_t maxit, int fuse_alpha, int64_t* iters);

/* ========================================================================================
 * LAGRANGE path: MCONTACT::LAGRANGE (MCONTACT.h:2847-3701) -- dual mortar basis (2894-2947),
 * nodal normal / tangent frames (2968-3038), normal-tangential mortar coupling (3040-3109),
 * static condensation of the non-mortar dofs (3281-3416) and the semi-smooth Newton active set
 * (stick / slip / open, 3637-3698); each Newton step's condensed system is solved on the device
 * by BiCGSTAB (MGPIS::BiCGSTAB_SOLV, MGPIS.h:350-432, stop ||r|| <= 1e-14 ||b||) preconditioned
 * with the MGPIS V-cycle of the hierarchy LAGRANGE builds for it (precType 1, 3419-3563) or the
 * diagonal (precType 2, the reference's Eigen::BiCGSTAB, 3565-3578).
 * ======================================================================================== */
typedef struct ddpca_lagrange* ddpca_lagrange_t;
int ddpca_lagrange_create(int64_t nsub, int64_t nint, ddpca_lagrange_t* out);
/* Subdomain tv as LAGRANGE reads it after TRANSFER / STIF_MATR / CONSTRAINT(precType == 1 ? 1 : -1)
 * (MCONTACT.h:2851-2860): nlev levels of mgpi.consStif K[l] (condensed, nfree[l] square), mgpi.realProl
 * P[l] (nfree[l+1] x nfree[l]), free_dof[l] (consOper[l]: condensed index -> position dof,
 * increasing, each level's a prefix of the next's), consForc; the node-id map
 * G = earlTran prolOper[maxiLeve] consOper[maxiLeve]^T (3 nnodes_all x nfree[nlev-1],
 * MCONTACT.h:3086-3088) and hanging[nnodes_all] (node id on level maxiLeve + 1, nodeLepo; may be
 * NULL: none). */
int ddpca_lagrange_set_subdomain(ddpca_lagrange_t h, int64_t tv, int nlev, const int64_t* nnodes,
                                 const int64_t* nfree, const int32_t* const* free_dof,
                                 const ddpca_csr_t* K, const ddpca_csr_t* P, const double* consForc,
                                 int64_t nnodes_all, const ddpca_csr_t* G, const uint8_t* hanging);
/* Interface ts: contBody {body0 (non-mortar), body1}, fricCoef (< 0 glued, 0 frictionless, > 0
 * Coulomb) and its integration points in ddpca_problem_set_ips's layout (node ids). */
int ddpca_lagrange_set_interface(ddpca_lagrange_t h, int64_t ts, int64_t body0, int64_t body1, double fric,
                                 int64_t n, const int64_t* node, const double* shap, const double* basis,
                                 const double* gap, const double* w);
/* Run the Newton loop; returns the reference's "Converge after tc-th iteration" tc (>= 0),
 * DDPCA_ENOCONV after max_newton steps, or another negative code.  opt: the V-cycle's smoother
 * settings (NULL: defaults); operators are kept fp64 (the system may be nonsymmetric). */
int64_t ddpca_lagrange_solve(ddpca_lagrange_t h, int device, int prec_type, const mgpis_options_t* opt,
                             int64_t max_newton);
/* Results of the last Newton step (doubles): "u" (index = subdomain: condensed displacement,
 * the subdomain's block of slidDisp, MCONTACT.h:3589), per interface (index = ts) over the
 * non-mortar nodes in the reference's (body, node) key order: "node" (node ids), "status"
 * (0 open, 1 slip, 2 stick: the active set the step solved with), "lambda" (3 per node,
 * resuLagr: normal, t1, t2), "wedi" (3 per node, nmnoWedi: weighted gap / relative
 * displacement); "solver_iters" and "changes" (per Newton step: BiCGSTAB iterations, seneNumb);
 * "solver_relres" (per Newton step: BiCGSTAB's recursive ||r|| / ||b|| at exit) and
 * "solver_breakdown" (0 converged to 1e-14, 1 rho = 0, 2 stopped at the attainable accuracy:
 * ||r|| <= 1e-12 ||b|| and flat over five iterations -- the singular frictionless systems).  A step
 * whose solve ends above 1e-10 makes ddpca_lagrange_solve return DDPCA_ENUMERIC.  "coarse_inverse"
 * (3 per Newton step: the dense coarse inverse taken -- 1 LU, kept only when ||A^-1 A - I||_inf
 * <= 1e-6, 2 SVD pseudo-inverse, -1 none (diagonal preconditioner) -- the LU residual measured
 * (inf when its pivot test failed) and the singular values the pseudo-inverse dropped).
 * Returns the count (copies min(count, cap) when out != NULL). */
int64_t ddpca_lagrange_get(ddpca_lagrange_t h, const char* what, int64_t index, double* out, int64_t cap);
int ddpca_lagrange_destroy(ddpca_lagrange_t h);

/* ========================================================================================
 * Result files in the reference's text formats (host only; std::scientific, precision 20,
 * width 30).  The reference rewrites resuDisp/resuCont on every ADMM iteration; a caller writes
 * them from mcontact_gpu_get / mcontact_gpu_monitor output when it wants them.
 * ======================================================================================== */
/* MULTIGRID::OUTP_SUB2 (MULTIGRID.h:1288-1307): one line "ux uy uz" per node of the nodal
 * displacement disp[3*nnodes]; the nrot nodes rot_node[k] (MULTIGRID::nodeRota) are rotated by
 * rot[9k..9k+8] (row-major) first. */
int ddpca_write_resuDisp(const char* path, const double* disp, int64_t nnodes, int64_t nrot,
                         const int64_t* rot_node, const double* rot);
/* MCONTACT::OUTPUT_PRTR (MCONTACT.h:97-123): fric == 0: one gamma_n per line; otherwise
 * "gamma_n  (gamma_1 t1 + gamma_2 t2)[0..2]  fricStat" per integration point, with gamma the
 * projected contact traction (3 per ip), stat the friction state (0 open, 1 slip, 2 stick;
 * mcontact_gpu_get "fricStat") and basis 9 doubles per ip (n, t1, t2; INTEGRAL_POINT::basiVect). */
int ddpca_write_resuCont(const char* path, double fric, int64_t nip, const double* gamma,
                         const int32_t* stat, const double* basis);
/* resuMoni.txt (MCONTACT.h:2502, 2742-2836): the rows of mcontact_gpu_monitor. */
int ddpca_write_resuMoni(const char* path, const double* rows, int64_t nrows, int64_t ncols);

#ifdef __cplusplus
}
#endif
#endif /* DDPCA_AMD_H */
