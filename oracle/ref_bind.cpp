// ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.
//
// Compiles the reference-side binding (oracle/ref_bind.hpp, quoted by INTEGRATION.md) against
// the reference's own headers and runs its host half: the reference builds the two-block
// contact problem and runs MCONTACT::ESTABLISH, the binding hands that output to
// libddpca_amd.so's operator-level builder, and the problem is read back through the C ABI and
// compared with the reference's matrices.  With "gpu", the device ADMM loop then runs on that
// problem (mcontact_gpu_*) and is compared with the reference's own CONTACT_ANALYSIS in the same
// process.  Prints JSON lines; exit code 0 = match.
//   ref_bind fric globLeve [gpu [muscSett]]
// "rot": a BEAM MULTIGRID with nodal rotations (nodeRota) on every fifth node, one rotation
// ("one") or a node-dependent one ("many"); the reference's CG_SOLV(1) vs mgpis_gpu_create_prol
// + mgpis_gpu_solve on the same hierarchy.  "roller": "one" plus a roller support on the tip face
// (local dof 0 of every tip node constrained): coarse nodes with partly constrained dofs, whose
// realProl rows/columns lack those dofs (consOper, MULTIGRID.h:1248).
//   ref_bind rot globLeve one|many|roller
#define HARNESS_NO_MAIN
#include "ref_harness.cpp"
#include "ref_bind.hpp"

namespace {

template <typename T>
std::vector<T> view(ddpca_problem_t p, const std::string& name, int64_t index, int64_t level) {
    const void* data = nullptr;
    int64_t n = 0;
    int dt = -1;
    ddpca_bind::check(ddpca_problem_view(p, name.c_str(), index, level, &data, &n, &dt));
    return std::vector<T>((const T*)data, (const T*)data + n);
}

ddpca_bind::SpMat csr_view(ddpca_problem_t p, const std::string& base, int64_t index, int64_t level) {
    auto shape = view<int64_t>(p, base + ":shape", index, level);
    auto ptr = view<int64_t>(p, base + ":ptr", index, level);
    auto col = view<int32_t>(p, base + ":col", index, level);
    auto val = view<double>(p, base + ":val", index, level);
    std::vector<Eigen::Triplet<double>> t;
    for (int64_t r = 0; r < shape[0]; ++r)
        for (int64_t k = ptr[r]; k < ptr[r + 1]; ++k) t.emplace_back(r, col[k], val[k]);
    ddpca_bind::SpMat m(shape[0], shape[1]);
    m.setFromTriplets(t.begin(), t.end());
    return m;
}

double maxabs(const ddpca_bind::SpMat& a) {
    double m = 0.0;
    for (int k = 0; k < a.outerSize(); ++k)
        for (ddpca_bind::SpMat::InnerIterator it(a, k); it; ++it) m = std::max(m, std::abs(it.value()));
    return m;
}

Eigen::Matrix3d axis_rotation(double ax, double ay, double az, double ang) {
    return Eigen::AngleAxisd(ang, Eigen::Vector3d(ax, ay, az).normalized()).toRotationMatrix();
}

int rot_mode(long gl, bool many, bool roller) {
    BEAM beam(0);
    beam.diviNumb = {8, 2, 2};
    beam.globLeve = gl;
    std::string log;
    MULTIGRID* gp = nullptr;
    harness::capture_iters([&] {
        beam.MESH_NODD(0);
        gp = &beam.multGrid[0];
        gp->TRANSFER();
        gp->STIF_MATR();
    }, &log);
    MULTIGRID& g = *gp;
    long nrot = 0;
    for (long ti = 0; ti < (long)g.nodeCoor.size(); ti += 5, ++nrot)
        g.nodeRota.emplace(ti, axis_rotation(1.0, 2.0, 3.0, many ? 0.3 + 0.001 * ti : 0.7));
    long nroll = 0;
    if (roller) {
        double xmax = -1e300;
        for (const auto& nc : g.nodeCoor) xmax = std::max(xmax, nc.second[0]);
        for (const auto& nc : g.nodeCoor)
            if (nc.second[0] >= xmax - 1e-9 * std::abs(xmax) && g.consDofv.emplace(3 * nc.first, 0.0).second) ++nroll;
    }
    harness::capture_iters([&] { g.CONSTRAINT(1); }, &log);
    long nblk = 0;  // realProl entries off w*I: the blocks the device runs as block entries
    for (long l = 0; l < g.mgpi.maxiLeve; ++l)
        for (int k = 0; k < g.mgpi.realProl[l].outerSize(); ++k)
            for (ddpca_bind::SpMat::InnerIterator it(g.mgpi.realProl[l], k); it; ++it)
                if (it.value() != 0.0 && it.value() != 1.0 && it.value() != 0.5 && it.value() != 0.25 &&
                    it.value() != 0.125)
                    ++nblk;
    Eigen::VectorXd x_ref;
    const long it_ref = harness::capture_iters([&] { g.mgpi.CG_SOLV(1, g.consForc, x_ref); });
    mgpis_options_t opt;
    mgpis_default_options(&opt);
    mgpis_t h = ddpca_bind::mgpis_create_prol(g, 0, &opt);
    Eigen::VectorXd x(g.consForc.size());
    int64_t it_gpu = 0;
    double rr = 0.0;
    ddpca_bind::check(mgpis_gpu_solve(h, g.consForc.data(), x.data(), 1, 1e-14, g.consForc.size(), &it_gpu, &rr));
    mgpis_gpu_destroy(h);
    const double dx = (x - x_ref).norm() / x_ref.norm();
    const bool ok = dx <= 1e-8 && nblk > 0 && (!roller || nroll > 0);
    std::printf("{\"rot_ok\": %s, \"n\": %ld, \"rotated_nodes\": %ld, \"rotated_prol_entries\": %ld, "
                "\"roller_dofs\": %ld, \"iters_ref\": %ld, \"iters_gpu\": %ld, \"x_rel\": %.3g}\n",
                ok ? "true" : "false", (long)x.size(), nrot, nblk, nroll, it_ref, (long)it_gpu, dx);
    return ok ? 0 : 1;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc >= 4 && std::string(argv[1]) == "rot")
        return rot_mode(std::stol(argv[2]), std::string(argv[3]) == "many", std::string(argv[3]) == "roller");
    if (argc < 3) { std::fprintf(stderr, "usage: ref_bind fric globLeve\n"); return 2; }
    MCONTACT mc;
    harness::twoblock_build(mc, std::stod(argv[1]), std::stol(argv[2]));
    if (argc > 4 && std::stol(argv[4]) != 0) {  // coarse space: 2 interface-eliminated (BLOCK.h:38-41), 1 LATIN
        mc.muscSett = std::stol(argv[4]);
        mc.doleMcsc.assign(mc.multGrid.size(), 1);
    }
    std::string log;
    harness::capture_iters([&] { mc.ESTABLISH(); }, &log);
    ddpca_problem_t p = ddpca_bind::from_reference(mc);
    double dK = 0.0, dP = 0.0, dF = 0.0, dOp = 0.0;
    for (size_t tv = 0; tv < mc.multGrid.size(); ++tv) {
        MULTIGRID& g = mc.multGrid[tv];
        for (long l = 0; l <= g.mgpi.maxiLeve; ++l)
            dK = std::max(dK, maxabs(csr_view(p, "K", tv, l) - g.mgpi.consStif[l]) / maxabs(g.mgpi.consStif[l]));
        for (long l = 0; l < g.mgpi.maxiLeve; ++l)
            dP = std::max(dP, maxabs(csr_view(p, "P", tv, l) - g.mgpi.realProl[l]));
        auto f = view<double>(p, "consForc", tv, 0);
        for (long i = 0; i < g.consForc.size(); ++i) dF = std::max(dF, std::abs(f[i] - g.consForc(i)));
    }
    const char* names[7] = {"inpoLagr", "pemaInpo_r", "systTran", "systTran_pena", "inteMass", "inteMass_pena",
                            "inteInpo"};
    for (size_t ts = 0; ts < mc.searCont.size(); ++ts)
        for (int s = 0; s < 2; ++s) {
            const auto& E = mc.multGrid[mc.contBody[ts][s]].earlTran;
            const ddpca_bind::SpMat ref[7] = {mc.inpoLagr[ts][s], mc.pemaInpo_r[ts][s] * E,
                                              E.transpose() * mc.systTran[ts][s],
                                              E.transpose() * mc.systTran_pena[ts][s], mc.inteMass[ts][s],
                                              mc.inteMass_pena[ts][s], mc.inteInpo[ts][s]};
            for (int k = 0; k < 7; ++k)
                dOp = std::max(dOp, maxabs(csr_view(p, names[k], 2 * ts + s, 0) - ref[k]));
        }
    bool ok = dK <= 1e-15 && dP == 0.0 && dF == 0.0 && dOp == 0.0;
    std::printf("{\"ok\": %s, \"subdomains\": %zu, \"interfaces\": %zu, \"K_rel\": %.3g, \"P\": %.3g, "
                "\"consForc\": %.3g, \"iface_ops\": %.3g}\n",
                ok ? "true" : "false", mc.multGrid.size(), mc.searCont.size(), dK, dP, dF, dOp);
    if (ok && argc > 3 && std::string(argv[3]) == "gpu") {
        // the device ADMM loop on the reference-built problem vs the reference's own loop
        std::vector<int32_t> owner(mc.multGrid.size(), 0);
        mcontact_t h = nullptr;
        ddpca_bind::check(mcontact_gpu_create(p, 0, 0, 1, owner.data(), nullptr, &h));
        const int64_t n_gpu = mcontact_gpu_iterate(h, 3000, 1);
        ddpca_bind::check((int)std::min<int64_t>(n_gpu, 0));
        harness::capture_iters([&] { mc.CONTACT_ANALYSIS(); }, &log);
        double du = 0.0;
        for (size_t tv = 0; tv < mc.multGrid.size(); ++tv) {
            const MULTIGRID& g = mc.multGrid[tv];
            Eigen::VectorXd u_pos(g.earlTran.cols());
            ddpca_bind::check((int)std::min<int64_t>(mcontact_gpu_get(h, "resuDisp", tv, u_pos.data(), u_pos.size()), 0));
            const Eigen::VectorXd u = g.earlTran * u_pos;  // position order -> node-id order (OUTP_SUB1)
            du = std::max(du, (u - mc.resuDisp[tv]).norm() / mc.resuDisp[tv].norm());
        }
        mcontact_gpu_destroy(h);
        const bool ok2 = std::abs(n_gpu - mc.iterNumbReco) <= 1 && du <= 1e-6;
        std::printf("{\"gpu_ok\": %s, \"iters_gpu\": %ld, \"iters_ref\": %ld, \"resuDisp_rel\": %.3g}\n",
                    ok2 ? "true" : "false", (long)n_gpu, (long)mc.iterNumbReco, du);
        ok = ok2;
    }
    ddpca_problem_destroy(p);
    return ok ? 0 : 1;
}
