// ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.
//
// Known-answer check on the reference's own TORSION example (examples/TORSION.h): a hollow
// shaft under an end torque, whose analytic end-face displacement is T*l/(G*I_p)*R =
// 1.159111630361142e-06 (TORSION.h:49).  The reference builds the {1,2,2}-subdomain DD problem
// (globHomo levels, muscSett = 2 interface-eliminated coarse space, TORSION.h:39) and runs its
// own CONTACT_ANALYSIS; oracle/ref_bind.hpp then hands the same ESTABLISH / MULTISCALE_1 output
// to the device and the device ADMM loop runs.  Prints one JSON line on stderr:
// iterations (device, reference), max nodal |u| (device, reference), resuDisp difference.
// dole = -1: doleMcsc = the fine level of every subdomain, so globCoup_1 has every free dof
// (126,750 rows at globHomo 2 >= DIRE_MAXI) and the reference solves it with its DOUBLE_M_1 MGPIS
// (MCONTACT.h:1857-1865, 2303-2341, 2593-2594) -- as the device does above that size.
// musc = 1: the LATIN coarse space instead (globCoup, DOUBLE_M past the same row count).
// ranks = N > 1: the same problem on N device ranks of one process (subdomain tv on rank tv % N,
// in-process transport) against a single-rank run of the same options (oracle/ref_ranks.hpp):
// BASELINE config 4's 4 subdomains on 4 ranks.
//   ref_torsion globHomo [dole] [musc] [ranks]
#include <unistd.h>

#include <cmath>
#include <cstdio>

#include "examples/TORSION.h"
#include "ref_bind.hpp"
#include "ref_ranks.hpp"

int main(int argc, char** argv) {
    const long gh = argc > 1 ? std::atol(argv[1]) : 2;
    const long dole = argc > 2 ? std::atol(argv[2]) : 1;
    const long musc = argc > 3 ? std::atol(argv[3]) : 2;
    const int nranks = argc > 4 ? std::atoi(argv[4]) : 1;
    const int saved = dup(1);
    if (!std::freopen("/dev/null", "w", stdout)) return 2;  // the reference's progress output
    TORSION t(1);
    t.domaNumb = {1, 2, 2};
    t.globHomo = gh;
    t.doleMcsc.assign(4, 1);
    t.ESTA_SURF();
    t.MESH_DD();
    if (dole < 0) t.doleMcsc.assign(4, t.multGrid[0].mgpi.maxiLeve);
    t.muscSett = musc;
    t.SOLVE_DD(1);  // ESTABLISH + the reference's CONTACT_ANALYSIS
    std::fflush(stdout);
    dup2(saved, 1);
    ddpca_problem_t p = ddpca_bind::from_reference(t);
    std::vector<int32_t> owner(t.multGrid.size(), 0);
    mcontact_t h = nullptr;
    ddpca_bind::check(mcontact_gpu_create(p, 0, 0, 1, owner.data(), nullptr, &h));
    const int64_t n_gpu = mcontact_gpu_iterate(h, 3000, 1);
    ddpca_bind::check((int)std::min<int64_t>(n_gpu, 0));
    double du = 0.0, umax_gpu = 0.0, umax_ref = 0.0;
    for (size_t tv = 0; tv < t.multGrid.size(); ++tv) {
        const MULTIGRID& g = t.multGrid[tv];
        Eigen::VectorXd u_pos(g.earlTran.cols());
        ddpca_bind::check((int)std::min<int64_t>(mcontact_gpu_get(h, "resuDisp", tv, u_pos.data(), u_pos.size()), 0));
        const Eigen::VectorXd u = g.earlTran * u_pos;  // position order -> node-id order (OUTP_SUB1)
        du = std::max(du, (u - t.resuDisp[tv]).norm() / t.resuDisp[tv].norm());
        for (long i = 0; i < u.size() / 3; ++i) {
            umax_gpu = std::max(umax_gpu, u.segment<3>(3 * i).norm());
            umax_ref = std::max(umax_ref, t.resuDisp[tv].segment<3>(3 * i).norm());
        }
    }
    const std::string alt = ddpca_ranks::coarse_alt(p, (int64_t)t.multGrid.size(), h, n_gpu);
    mcontact_gpu_destroy(h);
    std::string ranks = "null";
    if (nranks > 1) {
        std::vector<int32_t> ow(t.multGrid.size());
        for (size_t tv = 0; tv < ow.size(); ++tv) ow[tv] = (int32_t)(tv % nranks);
        std::vector<std::array<long, 2>> body;
        for (size_t ts = 0; ts < t.searCont.size(); ++ts) body.push_back({(long)t.contBody[ts][0], (long)t.contBody[ts][1]});
        mgpis_options_t o;
        mgpis_default_options(&o);
        o.coarse_level = 0;  // pinned: the automatic level depends on the subdomains per rank
        ranks = ddpca_ranks::compare(p, ow, nranks, (int64_t)t.multGrid.size(), (int64_t)t.searCont.size(), body, &o);
    }
    ddpca_problem_destroy(p);
    std::fprintf(stderr,
                 "{\"coarse_alt\": %s, \"ranks\": %s, \"iters_gpu\": %ld, \"iters_ref\": %ld, \"umax_gpu\": %.12g, \"umax_ref\": %.12g, "
                 "\"analytic\": 1.159111630361142e-06, \"resuDisp_rel\": %.3g, \"coarse_rows\": %ld, \"dofs\": %ld, \"interfaces\": %ld}\n",
                 alt.c_str(), ranks.c_str(), (long)n_gpu, (long)t.iterNumbReco, umax_gpu, umax_ref, du, (long)(musc == 1 ? t.globCoup.rows() : t.globCoup_1.rows()),
                 (long)[&] { long n = 0; for (auto& g : t.multGrid) n += g.mgpi.consStif[g.mgpi.maxiLeve].rows(); return n; }(),
                 (long)t.searCont.size());
    return 0;
}
