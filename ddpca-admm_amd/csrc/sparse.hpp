// Host-side sparse containers for the MULTIGRID operator pipeline.
//
// The reference stores every operator as Eigen::SparseMatrix<double,RowMajor> (scalar CSR,
// int32 indices: PREP.h:107-113, MGPIS.h:13-33).  Elasticity operators here are 3x3-node-block
// structured, so the host keeps them as BSR3 (one int32 column index per 3x3 block) and only
// expands to scalar CSR at the reference-compatible C-ABI boundary (include/ddpca_amd.h).
#pragma once
#include <array>
#include <cstdint>
#include <vector>

namespace ddpca {

// Scalar CSR, int64 row pointer, int32 columns (reference layout: Eigen RowMajor, int index).
struct Csr {
    int64_t nrow = 0, ncol = 0;
    std::vector<int64_t> ptr;
    std::vector<int32_t> col;
    std::vector<double> val;
    int64_t nnz() const { return (int64_t)col.size(); }
};

// 3x3 block CSR: block row i / block col j = node i / node j; val holds 9 doubles per block,
// row-major (dof 3i+a, 3j+b) at val[9*k + 3*a + b].  Columns sorted within a row.
struct Bsr3 {
    int64_t nb = 0, mb = 0;  // block rows / block cols (nodes)
    std::vector<int64_t> ptr;
    std::vector<int32_t> col;
    std::vector<double> val;
    int64_t nnzb() const { return (int64_t)col.size(); }
    const double* block(int64_t k) const { return &val[9 * k]; }
    double* block(int64_t k) { return &val[9 * k]; }
    // y = A x (dof vectors of length 3*mb / 3*nb)
    void apply(const double* x, double* y) const;
};

// Scalar prolongation stencil between node levels (MULTIGRID::scalProl, MULTIGRID.h:911-946):
// rows = fine nodes, cols = coarse nodes; first `ncoarse` rows are the identity (level-ordered
// numbering keeps every coarse node at the same index on the finer level).
struct Stencil {
    int64_t nf = 0, nc = 0;
    std::vector<int64_t> ptr;
    std::vector<int32_t> col;
    std::vector<double> w;
    // entries whose 3x3 block is not w*I (nodal rotations, MULTIGRID.h:1141-1181): entry index
    // into col/w (its w is 0) and the full block, row-major, 9 per entry; empty when P = S (x) I3
    std::vector<int64_t> bent;
    std::vector<double> bval;
};

// C = P^T A P for a BSR3 A on the fine nodes and P = S (x) I3 (Galerkin product,
// MULTIGRID.h:1182-1184), S's block entries (rotated nodes) taken as their 3x3 blocks.
Bsr3 galerkin_rap(const Bsr3& A, const Stencil& S);

// Expand to scalar CSR keeping only dofs with keep[dof] != 0 (consOper * A * consOper^T,
// MULTIGRID.h:1213-1227).  free_index[dof] = condensed index or -1.
Csr condense(const Bsr3& A, const std::vector<int32_t>& free_index, int64_t nfree);

// Inverse direction, from the reference's layout: condensed CSR (consStif[l], nfree rows) and
// its free-dof map (condensed row -> nodal dof 3*node + comp) -> node-block BSR3 on nn nodes
// whose constrained rows/cols are zero (the device masks them to identity); every node keeps
// its diagonal block.
Bsr3 condensed_to_bsr3(int64_t nn, int64_t nfree, const int32_t* free_dof, const int64_t* ptr, const int32_t* col,
                       const double* val);

Stencil make_stencil(int64_t nf, int64_t nc, const int64_t* ptr, const int32_t* col, const double* w);

// Node stencil of the reference's realProl[l] = consOper[l+1] prolOper[l] consOper[l]^T
// (MULTIGRID.h:1141-1181, 1246-1249) given as condensed CSR (nfree_f x nfree_c): every
// (fine node, coarse node) block whose free part is w*I becomes a scalar entry, any other block
// (rotated nodes, nodeRota) a block entry.  Coarse nodes keep the identity row.
Stencil prol_to_stencil(int64_t nf, int64_t nc, int64_t nfree_f, const int32_t* free_f, const int32_t* free_c,
                        const int64_t* ptr, const int32_t* col, const double* val);

}  // namespace ddpca
