// The reference's result files, written from host arrays (no GPU needed): resuDisp_<tv>.txt
// (MULTIGRID::OUTP_SUB2, MULTIGRID.h:1288-1307), resuCont_<ts>.txt (MCONTACT::OUTPUT_PRTR,
// MCONTACT.h:97-123) and resuMoni.txt (the rows MCONTACT::MONITOR appends, MCONTACT.h:2742-2836).
// The reference streams with std::scientific, setprecision(20), setw(30) (setw(10) for the
// friction state); printf's "%30.20e" / "%10d" produce the same characters.  The reference
// rewrites resuDisp/resuCont on every ADMM iteration; here the caller writes them when it wants
// them (the content equals the reference's final files).
#include <cmath>
#include <cstdio>
#include <map>
#include <memory>

#include "../../include/ddpca_amd.h"
#include "common.hpp"

using namespace ddpca;

namespace {

struct File {
    std::FILE* f;
    explicit File(const char* path) : f(path ? std::fopen(path, "w") : nullptr) {
        if (!f) throw ApiError(DDPCA_EINVAL, std::string("cannot open for writing: ") + (path ? path : "(null)"));
    }
    ~File() {
        if (f) std::fclose(f);
    }
    void num(double v) { std::fprintf(f, "%30.20e", v); }
    void end() { std::fputc('\n', f); }
};

}  // namespace

extern "C" {

int ddpca_write_resuDisp(const char* path, const double* disp, int64_t nnodes, int64_t nrot, const int64_t* rot_node,
                         const double* rot) {
    return guarded([&] {
        if (nnodes < 0 || (nnodes > 0 && !disp) || nrot < 0 || (nrot > 0 && (!rot_node || !rot)))
            throw ApiError(DDPCA_EINVAL, "ddpca_write_resuDisp: bad arguments");
        std::map<int64_t, const double*> nodeRota;  // MULTIGRID::nodeRota
        for (int64_t k = 0; k < nrot; ++k) nodeRota[rot_node[k]] = rot + 9 * k;
        File out(path);
        for (int64_t i = 0; i < nnodes; ++i) {
            double d[3] = {disp[3 * i], disp[3 * i + 1], disp[3 * i + 2]};
            const auto it = nodeRota.find(i);
            if (it != nodeRota.end()) {
                const double* R = it->second;
                const double e[3] = {d[0], d[1], d[2]};
                for (int a = 0; a < 3; ++a) d[a] = R[3 * a] * e[0] + R[3 * a + 1] * e[1] + R[3 * a + 2] * e[2];
            }
            for (int a = 0; a < 3; ++a) out.num(d[a]);
            out.end();
        }
    });
}

int ddpca_write_resuCont(const char* path, double fric, int64_t nip, const double* gamma, const int32_t* stat,
                         const double* basis) {
    return guarded([&] {
        if (nip < 0 || (nip > 0 && !gamma)) throw ApiError(DDPCA_EINVAL, "ddpca_write_resuCont: bad arguments");
        if (fric != 0.0 && nip > 0 && (!stat || !basis))
            throw ApiError(DDPCA_EINVAL, "ddpca_write_resuCont: fricCoef != 0 needs the friction state and the ip basis");
        File out(path);
        for (int64_t q = 0; q < nip; ++q) {
            if (fric == 0.0) {
                out.num(gamma[q]);
                out.end();
                continue;
            }
            // traction along the tangents: gamma_1 t1 + gamma_2 t2 (basiVect[1], [2])
            const double* t1 = basis + 9 * q + 3;
            const double* t2 = basis + 9 * q + 6;
            out.num(gamma[3 * q]);
            for (int a = 0; a < 3; ++a) out.num(gamma[3 * q + 1] * t1[a] + gamma[3 * q + 2] * t2[a]);
            std::fprintf(out.f, "%10d", (int)stat[q]);
            out.end();
        }
    });
}

int ddpca_write_resuMoni(const char* path, const double* rows, int64_t nrows, int64_t ncols) {
    return guarded([&] {
        if (nrows < 0 || ncols < 0 || (nrows * ncols > 0 && !rows)) throw ApiError(DDPCA_EINVAL, "ddpca_write_resuMoni: bad arguments");
        File out(path);
        for (int64_t r = 0; r < nrows; ++r) {
            for (int64_t c = 0; c < ncols; ++c) out.num(rows[r * ncols + c]);
            out.end();
        }
    });
}

}  // extern "C"
