// ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.
//
// Known-answer check on the reference's own BLOCK example (examples/BLOCK.h): stacked blocks
// under a uniform 1e7 Pa top load, so the contact pressure between them is the patch-test value
// 1e7 (BLOCK.h:46 comment).  The reference builds the domaNumb {1,1,1} problem at the
// given globLeve with the given muscSett and runs its own CONTACT_ANALYSIS; oracle/ref_bind.hpp
// hands the same operators to the device, whose ADMM loop then runs.  One JSON line on stderr:
// iterations, resuDisp difference, and per interface the device's mean/min/max normal pressure.
//   ref_block globLeve muscSett
#include <unistd.h>

#include <cstdio>

#include "examples/BLOCK.h"
#include "ref_bind.hpp"
#include "ref_ranks.hpp"

int main(int argc, char** argv) {
    const long gl = argc > 1 ? std::atol(argv[1]) : 1;
    const long musc = argc > 2 ? std::atol(argv[2]) : 1;
    const int saved = dup(1);
    if (!std::freopen("/dev/null", "w", stdout)) return 2;  // the reference's progress output
    BLOCK b;
    b.domaNumb = {1, 1, 1};
    b.globLeve = gl;
    b.muscSett = musc;
    b.doleMcsc.assign(3 * 1 + 6, 1);
    b.ESTA_SURF();
    b.SOLVE(1);  // MESH, ESTABLISH and the reference's CONTACT_ANALYSIS
    std::fflush(stdout);
    dup2(saved, 1);
    ddpca_problem_t p = ddpca_bind::from_reference(b);
    std::vector<int32_t> owner(b.multGrid.size(), 0);
    mcontact_t h = nullptr;
    ddpca_bind::check(mcontact_gpu_create(p, 0, 0, 1, owner.data(), nullptr, &h));
    const int64_t n_gpu = mcontact_gpu_iterate(h, 3000, 1);
    ddpca_bind::check((int)std::min<int64_t>(n_gpu, 0));
    double du = 0.0;
    for (size_t tv = 0; tv < b.multGrid.size(); ++tv) {
        const MULTIGRID& g = b.multGrid[tv];
        Eigen::VectorXd u_pos(g.earlTran.cols());
        ddpca_bind::check((int)std::min<int64_t>(mcontact_gpu_get(h, "resuDisp", tv, u_pos.data(), u_pos.size()), 0));
        const Eigen::VectorXd u = g.earlTran * u_pos;
        du = std::max(du, (u - b.resuDisp[tv]).norm() / b.resuDisp[tv].norm());
    }
    std::string itf = "[";
    std::vector<double> gam(1 << 22);
    for (size_t ts = 0; ts < b.searCont.size(); ++ts) {
        const int64_t n = mcontact_gpu_get(h, "inpoGamm", ts, gam.data(), (int64_t)gam.size());
        ddpca_bind::check((int)std::min<int64_t>(n, 0));
        const int comp = b.fricCoef[ts] == 0.0 ? 1 : 3;
        double s = 0.0, mn = 1e300, mx = -1e300;
        int64_t m = 0;
        for (int64_t i = 0; i < n / comp; ++i) {
            const double g = gam[comp * i];
            s += g;
            mn = std::min(mn, g);
            mx = std::max(mx, g);
            ++m;
        }
        char buf[160];
        std::snprintf(buf, sizeof(buf), "%s{\"ts\": %zu, \"nip\": %ld, \"mean\": %.9g, \"min\": %.9g, \"max\": %.9g}",
                      ts ? ", " : "", ts, (long)m, m ? s / m : 0.0, mn, mx);
        itf += buf;
    }
    itf += "]";
    const std::string alt = ddpca_ranks::coarse_alt(p, (int64_t)b.multGrid.size(), h, n_gpu);
    mcontact_gpu_destroy(h);
    ddpca_problem_destroy(p);
    std::fprintf(stderr, "{\"coarse_alt\": %s, \"iters_gpu\": %ld, \"iters_ref\": %ld, \"resuDisp_rel\": %.3g, \"interfaces\": %s}\n",
                 alt.c_str(), (long)n_gpu, (long)b.iterNumbReco, du, itf.c_str());
    return 0;
}
