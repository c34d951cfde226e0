// ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.
//
// Multi-rank check of an established device problem on ONE GPU: the same problem on `owners`'
// ranks, each rank a device handle of this process connected to the others by the in-process
// transport (mcontact_gpu_comm_local: RCCL's matching rules -- grouped sends and receives paired per
// peer in issue order -- on host-staged copies), every rank's ADMM loop on its own host thread.
// Compared with a single-rank device run of the same problem and options: iteration counts,
// resuMoni rows (relative, floor 1e-12 of the column's largest value), resuDisp of every subdomain
// (its owner's copy) and the projected gamma of every interface (the first side owner's copy).
// The reference keeps all subdomains in one process (MCONTACT.h:2511-2537, 2629-2704); the device
// distributes them, so this is what stands between the one-GPU tests and an 8-GPU run.
#pragma once
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "ddpca_amd.h"

namespace ddpca_ranks {

inline void check(int rc) {
    if (rc < 0) throw std::runtime_error(std::string("libddpca_amd: ") + ddpca_last_error());
}

// body[ts] = {contBody[ts][0], contBody[ts][1]}; returns one JSON object
inline std::string compare(ddpca_problem_t p, const std::vector<int32_t>& owners, int nranks, int64_t nsub, int64_t nint,
                           const std::vector<std::array<long, 2>>& body, const mgpis_options_t* opt, int64_t maxit = 3000) {
    const int64_t ncol = 2 * nsub + 8 * nint + 2;
    std::vector<int32_t> zero(nsub, 0);
    mcontact_t h1 = nullptr;
    check(mcontact_gpu_create(p, 0, 0, 1, zero.data(), opt, &h1));
    const int64_t n1 = mcontact_gpu_iterate(h1, maxit, 1);
    check((int)std::min<int64_t>(n1, 0));
    const int64_t rows1 = mcontact_gpu_monitor(h1, nullptr, 0);
    std::vector<double> moni1(rows1 * ncol);
    mcontact_gpu_monitor(h1, moni1.data(), rows1);

    std::vector<mcontact_t> hr(nranks, nullptr);
    for (int r = 0; r < nranks; ++r) check(mcontact_gpu_create(p, 0, r, nranks, owners.data(), opt, &hr[r]));
    check(mcontact_gpu_comm_local(hr.data(), nranks));
    std::vector<int64_t> nr(nranks, 0);
    std::vector<int> ck(nranks, 0);
    std::vector<std::string> msg(nranks);  // the library's last error is per thread
    {
        std::vector<std::thread> th;
        for (int r = 0; r < nranks; ++r)
            th.emplace_back([&, r] {
                ck[r] = mcontact_gpu_comm_check(hr[r], 4096);  // the transport itself first
                nr[r] = ck[r] < 0 ? ck[r] : mcontact_gpu_iterate(hr[r], maxit, 1);
                if (nr[r] < 0) msg[r] = std::string(ck[r] < 0 ? "comm_check: " : "iterate: ") + ddpca_last_error();
            });
        for (auto& t : th) t.join();
    }
    for (int r = 0; r < nranks; ++r)
        if (nr[r] < 0) throw std::runtime_error("libddpca_amd: rank " + std::to_string(r) + " " + msg[r]);
    // resuMoni (MCONTACT.h:2742-2836): the odd columns are squared norms of the iterates (||u||^2,
    // ||aux||^2, ...), the even ones squared differences of successive iterates -- late in the run
    // differences of nearly equal vectors, whose relative error grows as (|u| eps / |du|)^2: the two
    // kinds are reported apart (dm: norms, dd: differences)
    double dm = 0.0, dd = 0.0, du = 0.0, dg = 0.0;
    for (int r = 0; r < nranks; ++r) {
        const int64_t rows = mcontact_gpu_monitor(hr[r], nullptr, 0);
        std::vector<double> m(rows * ncol);
        mcontact_gpu_monitor(hr[r], m.data(), rows);
        if (rows != rows1) dm = dd = 1e300;
        for (int64_t j = 0; j < ncol && rows == rows1; ++j) {
            double scale = 0.0;
            for (int64_t k = 0; k < rows; ++k) scale = std::max(scale, std::abs(moni1[k * ncol + j]));
            double& d = (j % 2 == 1) ? dm : dd;
            for (int64_t k = 0; k < rows; ++k) {
                const double a = m[k * ncol + j], b = moni1[k * ncol + j];
                d = std::max(d, std::abs(a - b) / (std::abs(b) + 1e-12 * scale + 1e-300));
            }
        }
    }
    for (int64_t tv = 0; tv < nsub; ++tv) {
        const int64_t n = mcontact_gpu_get(h1, "resuDisp", tv, nullptr, 0);
        std::vector<double> a(n), b(n);
        mcontact_gpu_get(h1, "resuDisp", tv, b.data(), n);
        check((int)std::min<int64_t>(mcontact_gpu_get(hr[owners[tv]], "resuDisp", tv, a.data(), n), 0));
        double d = 0.0, s = 0.0;
        for (int64_t i = 0; i < n; ++i) d += (a[i] - b[i]) * (a[i] - b[i]), s += b[i] * b[i];
        du = std::max(du, std::sqrt(d / std::max(s, 1e-300)));
    }
    int64_t cross = 0;
    for (int64_t ts = 0; ts < nint; ++ts) {
        const int r = owners[body[ts][0]];
        cross += owners[body[ts][0]] != owners[body[ts][1]];
        const int64_t n = mcontact_gpu_get(h1, "inpoGamm", ts, nullptr, 0);
        std::vector<double> a(n), b(n);
        mcontact_gpu_get(h1, "inpoGamm", ts, b.data(), n);
        check((int)std::min<int64_t>(mcontact_gpu_get(hr[r], "inpoGamm", ts, a.data(), n), 0));
        double gm = 0.0, d = 0.0;
        for (int64_t i = 0; i < n; ++i) gm = std::max(gm, std::abs(b[i])), d = std::max(d, std::abs(a[i] - b[i]));
        dg = std::max(dg, gm > 0 ? d / gm : d);
    }
    for (auto& x : hr) mcontact_gpu_destroy(x);
    mcontact_gpu_destroy(h1);
    std::string own, its;
    for (size_t tv = 0; tv < owners.size(); ++tv) own += (tv ? ", " : "") + std::to_string(owners[tv]);
    for (int r = 0; r < nranks; ++r) its += std::to_string(nr[r]) + (r + 1 < nranks ? ", " : "");
    char buf[512];
    std::snprintf(buf, sizeof(buf),
                  "{\"nranks\": %d, \"owners\": [%s], \"cross_interfaces\": %ld, \"iters_1rank\": %ld, \"iters\": [%s], "
                  "\"moni_rel\": %.3g, \"moni_diff_rel\": %.3g, \"resuDisp_rel\": %.3g, \"gamma_rel\": %.3g}",
                  nranks, own.c_str(), (long)cross, (long)n1, its.c_str(), dm, dd, du, dg);
    return buf;
}

// The same problem solved with the coarse space's other solve (the dense inverse <-> the
// multigrid solve of DOUBLE_M / DOUBLE_M_1, switched by the dense-inverse memory budget
// DDPCA_COARSE_DENSE_MB): iterations and resuDisp (position order) against the first run's.
// Returns a JSON object; "null" when the first run had no coarse space or its multigrid solve was
// forced by the row count (DIRE_MAXI), where the dense inverse is not available.
inline std::string coarse_alt(ddpca_problem_t p, int64_t nsub, mcontact_t h0, int64_t n0, int64_t maxit = 3000) {
    int64_t cs0[4] = {0, 0, 0, 0};
    check((int)std::min<int64_t>(mcontact_gpu_get(h0, "coarse_solve", 0, cs0, 4), 0));
    if (cs0[0] == 0 || (cs0[1] == 1 && cs0[0] >= 120000)) return "null";
    const char* old = std::getenv("DDPCA_COARSE_DENSE_MB");
    const std::string keep = old ? old : "";
    setenv("DDPCA_COARSE_DENSE_MB", cs0[1] ? "1e9" : "0", 1);
    std::vector<int32_t> zero(nsub, 0);
    mcontact_t h = nullptr;
    const int rc = mcontact_gpu_create(p, 0, 0, 1, zero.data(), nullptr, &h);
    if (old) setenv("DDPCA_COARSE_DENSE_MB", keep.c_str(), 1);
    else unsetenv("DDPCA_COARSE_DENSE_MB");
    check(rc);
    int64_t cs1[4] = {0, 0, 0, 0};
    check((int)std::min<int64_t>(mcontact_gpu_get(h, "coarse_solve", 0, cs1, 4), 0));
    const int64_t n1 = mcontact_gpu_iterate(h, maxit, 1);
    check((int)std::min<int64_t>(n1, 0));
    double du = 0.0;
    for (int64_t tv = 0; tv < nsub; ++tv) {
        const int64_t n = mcontact_gpu_get(h0, "resuDisp", tv, nullptr, 0);
        std::vector<double> a(n), b(n);
        check((int)std::min<int64_t>(mcontact_gpu_get(h0, "resuDisp", tv, b.data(), n), 0));
        check((int)std::min<int64_t>(mcontact_gpu_get(h, "resuDisp", tv, a.data(), n), 0));
        double d = 0.0, s = 0.0;
        for (int64_t i = 0; i < n; ++i) d += (a[i] - b[i]) * (a[i] - b[i]), s += b[i] * b[i];
        du = std::max(du, std::sqrt(d / std::max(s, 1e-300)));
    }
    mcontact_gpu_destroy(h);
    char buf[320];
    std::snprintf(buf, sizeof(buf),
                  "{\"rows\": %ld, \"first_mg\": %ld, \"first_dense_bytes\": %ld, \"alt_mg\": %ld, \"alt_fallback\": %ld, \"iters_first\": %ld, "
                  "\"iters_alt\": %ld, \"resuDisp_rel\": %.3g}",
                  (long)cs0[0], (long)cs0[1], (long)cs0[2], (long)cs1[1], (long)cs1[3], (long)n0, (long)n1, du);
    return buf;
}

}  // namespace ddpca_ranks
