// ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.
//
// The reference's own CYLINDER example (examples/CYLINDER_1.h: a stack of four cylinder bodies
// in Hertz contact, locally refined towards the contact lines -- hanging nodes on a level past
// the MGPIS hierarchy, MULTIGRID.h:836-848 -- contact search on the curved surfaces, LATIN-type
// coarse space muscSett = 1 with doleMcsc = 2).  The reference builds it at a reduced size and
// runs its own CONTACT_ANALYSIS; oracle/ref_bind.hpp hands the same operators (with the hanging
// level, ddpca_problem_set_hanging) to the device, whose ADMM loop then runs.  One JSON line on
// stderr: iterations, resuDisp difference (node-id order, every node incl. the hanging ones), the
// resuMoni trajectory and the contact pressures against the reference's last resuCont files.
// "native": every subdomain's operators come from the library's own pipeline on the element tree
// (ddpca_multigrid_*: TRANSFER with the hanging level, PATCH, STIF_MATR + the contact systMass,
// CONSTRAINT(1)) instead of the reference's MULTIGRID; the interface and coarse operators stay the
// reference's.  owners (e.g. 0011): the same problem on two device ranks in one process, connected
// by the in-process test transport (mcontact_gpu_comm_local), subdomain tv owned by rank
// owners[tv]: rank-local batches with the hanging level, the gamma halves of the cross-rank
// curved contacts exchanged, the LATIN coarse space's operator rows filled by rank 0 and summed,
// the MONITOR all-reduce -- compared with the single-rank device run (iterations equal, resuMoni
// 1e-8, displacements 1e-8, contact tractions 1e-7 of the largest).
//   ref_cylinder copyNumb locaLeve globInho bandWidt [variants: ref,native,ref-mc,native-mc] [owners] [noref]
#include <unistd.h>

#include <cstdio>
#include <cstdlib>
#include <memory>
#include <thread>
#include <fstream>
#include <sstream>

#include "examples/CYLINDER_1.h"
#include "ref_bind.hpp"
#include "ref_ranks.hpp"

namespace {

std::vector<std::vector<double>> read_rows(const std::string& path) {
    std::vector<std::vector<double>> rows;
    std::ifstream f(path);
    std::string line;
    while (std::getline(f, line)) {
        std::istringstream is(line);
        std::vector<double> r;
        double v;
        while (is >> v) r.push_back(v);
        if (!r.empty()) rows.push_back(r);
    }
    return rows;
}

}  // namespace

int main(int argc, char** argv) {
    const long copyNumb = argc > 1 ? std::atol(argv[1]) : 1;
    const long locaLeve = argc > 2 ? std::atol(argv[2]) : 4;
    const long globInho = argc > 3 ? std::atol(argv[3]) : 2;
    const double bandWidt = argc > 4 ? std::atof(argv[4]) : 2.0e-4;
    const int saved = dup(1);
    if (!std::freopen("/dev/null", "w", stdout)) return 2;  // the reference's progress output
    CYLINDER_1 c;  // creates ./Cylinder/ for the reference's result files
    c.copyNumb = copyNumb;
    c.locaLeve = locaLeve;
    c.globInho = globInho;
    c.bandWidt = bandWidt;
    // noref (after the owners): the two-rank comparison alone -- the reference builds the problem
    // (MESH, contact search, ESTABLISH) but does not run its CONTACT_ANALYSIS, whose answers
    // test_cylinder_known_answer checks
    const bool noref = argc > 7 && std::string(argv[7]) == "noref";
    c.SOLVE(noref ? 0 : 1);  // MESH, contact search, ESTABLISH (and the reference's CONTACT_ANALYSIS)
    std::fflush(stdout);
    dup2(saved, 1);
    long nhang = 0, nnodes = 0;
    for (auto& g : c.multGrid) {
        nnodes += (long)g.nodeCoor.size();
        nhang += (long)g.leveNode[g.mgpi.maxiLeve + 1].size();
    }
    // variants (argv[5], comma-separated; one JSON line each, on the same reference run):
    // ref / native = the operators' source (the reference's MULTIGRID or the library's own pipeline
    // on the element trees), "-mc" = the headline's V-cycle (colour Gauss-Seidel on the fine level --
    // band mode where the fine level refines a band -- two block-Jacobi sweeps below, block-scaled
    // int8 copies) instead of the default block Jacobi; DDPCA_REF_OPTIONS=multicolour makes every
    // variant "-mc" (the single-variant form of earlier rounds)
    std::vector<std::string> variants;
    {
        std::string v = argc > 5 ? argv[5] : "ref";
        size_t a = 0;
        while (a <= v.size()) {
            const size_t b = std::min(v.find(',', a), v.size());
            if (b > a) variants.push_back(v.substr(a, b - a));
            a = b + 1;
        }
    }
    const char* oe = std::getenv("DDPCA_REF_OPTIONS");
    const bool mcol_env = oe && std::string(oe) == "multicolour";
    bool any_native = false;
    for (const auto& v : variants) {
        if (v != "ref" && v != "native" && v != "ref-mc" && v != "native-mc") {
            std::fprintf(stderr, "variant: ref, native, ref-mc or native-mc\n");
            return 2;
        }
        any_native |= v.rfind("native", 0) == 0;
    }
    std::unique_ptr<CYLINDER_1> trees;  // the same meshes again, before any TRANSFER / PATCH
    if (any_native) {
        if (!std::freopen("/dev/null", "w", stdout)) return 2;
        trees.reset(new CYLINDER_1);
        trees->copyNumb = copyNumb;
        trees->locaLeve = locaLeve;
        trees->globInho = globInho;
        trees->bandWidt = bandWidt;
        trees->MESH();
        std::fflush(stdout);
        dup2(saved, 1);
    }
    const auto ref_moni = noref ? std::vector<std::vector<double>>() : read_rows(DIRECTORY("resuMoni.txt"));
    std::vector<std::vector<std::vector<double>>> ref_cont;
    for (size_t ts = 0; ts < c.searCont.size() && !noref; ++ts)
        ref_cont.push_back(read_rows(DIRECTORY("resuCont_" + std::to_string(ts) + ".txt")));
    for (size_t vi = 0; vi < variants.size(); ++vi) {
        const bool native = variants[vi].rfind("native", 0) == 0;
        const bool mcol = mcol_env || variants[vi].size() > 3 && variants[vi].compare(variants[vi].size() - 3, 3, "-mc") == 0;
        double dK = 0.0;  // native: our consStif vs the reference's, relative to the level maximum
        ddpca_problem_t p = ddpca_bind::from_reference(c, [&](ddpca_problem_t prob, int64_t tv) {
            if (!native) return false;
            ddpca_bind::SpMat extra(3 * c.multGrid[tv].nodeCoor.size(), 3 * c.multGrid[tv].nodeCoor.size());
            for (size_t ts = 0; ts < c.searCont.size(); ++ts)
                for (int s = 0; s < 2; ++s)
                    if (c.contBody[ts][s] == tv) extra += c.systMass[ts][s];
            ddpca_multigrid_t h = ddpca_bind::tree_build(trees->multGrid[tv], &extra);
            ddpca_bind::check(ddpca_problem_set_subdomain_multigrid(prob, tv, h));
            ddpca_multigrid_destroy(h);
            const MULTIGRID& g = c.multGrid[tv];
            for (long l = 0; l <= g.mgpi.maxiLeve; ++l) {
                const ddpca_bind::SpMat K = ddpca_bind::problem_csr(prob, "K", tv, l);
                const ddpca_bind::SpMat D = K - g.mgpi.consStif[l];
                double m = 0.0, r = 0.0;
                for (int k = 0; k < D.outerSize(); ++k)
                    for (ddpca_bind::SpMat::InnerIterator it(D, k); it; ++it) m = std::max(m, std::abs(it.value()));
                for (int k = 0; k < g.mgpi.consStif[l].outerSize(); ++k)
                    for (ddpca_bind::SpMat::InnerIterator it(g.mgpi.consStif[l], k); it; ++it) r = std::max(r, std::abs(it.value()));
                dK = std::max(dK, m / r);
            }
            return true;
        });
        std::vector<int32_t> owner(c.multGrid.size(), 0);
        mcontact_t h = nullptr;
        mgpis_options_t opt;
        mgpis_default_options(&opt);
        if (mcol) {
            opt.smoother = 3;
            opt.nu = 2;
            opt.precond_fp32 = 3;
        }
        ddpca_bind::check(mcontact_gpu_create(p, 0, 0, 1, owner.data(), &opt, &h));
        int64_t gsr[3] = {0, 0, 0};
        ddpca_bind::check((int)std::min<int64_t>(mcontact_gpu_get(h, "gs_rows", 0, gsr, 3), 0));
        const int64_t n_gpu = noref ? 0 : mcontact_gpu_iterate(h, 3000, 1);
        ddpca_bind::check((int)std::min<int64_t>(n_gpu, 0));
        // displacements: position order (hanging level last) -> node-id order
        double du = 0.0;
        for (size_t tv = 0; tv < c.multGrid.size() && !noref; ++tv) {
            const MULTIGRID& g = c.multGrid[tv];
            Eigen::VectorXd u_pos(g.earlTran.cols());
            const int64_t n = mcontact_gpu_get(h, "resuDisp", tv, u_pos.data(), u_pos.size());
            ddpca_bind::check((int)std::min<int64_t>(n, 0));
            if (n != u_pos.size()) {
                std::fprintf(stderr, "resuDisp of %zu has %ld entries, expected %ld\n", tv, (long)n, (long)u_pos.size());
                return 1;
            }
            const Eigen::VectorXd u = g.earlTran * u_pos;
            du = std::max(du, (u - c.resuDisp[tv]).norm() / c.resuDisp[tv].norm());
        }
        // resuMoni rows (the reference's file, scientific 20 digits) vs the device's monitor rows
        const int64_t ncol = 2 * (int64_t)c.multGrid.size() + 8 * (int64_t)c.searCont.size() + 2;
        const int64_t nrows = mcontact_gpu_monitor(h, nullptr, 0);
        std::vector<double> moni(nrows * ncol);
        mcontact_gpu_monitor(h, moni.data(), nrows);
        double dmoni = 0.0;  // rows k <= 50, the columns of the squared norms (even columns), relative
        const int64_t kmax = std::min<int64_t>(std::min<int64_t>(50, nrows), (int64_t)ref_moni.size());
        for (int64_t k = 0; k < kmax; ++k)
            for (int64_t j = 1; j < ncol; j += 2) {  // odd columns: ||u||^2, ||aux||^2, ...: well scaled
                const double r = ref_moni[k][j], d = moni[k * ncol + j];
                if (r != 0.0) dmoni = std::max(dmoni, std::abs(d - r) / std::abs(r));
            }
        // contact pressures (frictionless: one gamma_n per ip) vs the reference's last resuCont
        std::string itf = "[";
        std::vector<double> gam(1 << 22);
        double dp_all = 0.0;
        for (size_t ts = 0; ts < c.searCont.size() && !noref; ++ts) {
            const int64_t n = mcontact_gpu_get(h, "inpoGamm", ts, gam.data(), (int64_t)gam.size());
            ddpca_bind::check((int)std::min<int64_t>(n, 0));
            const auto& ref = ref_cont[ts];
            const int comp = c.fricCoef[ts] == 0.0 ? 1 : 3;
            double pmax = 0.0, dp = 0.0, gmax = 0.0;
            int64_t active = 0;
            for (size_t i = 0; i < ref.size(); ++i) pmax = std::max(pmax, ref[i][0]);
            for (int64_t i = 0; i < n / comp && i < (int64_t)ref.size(); ++i) {
                const double g = gam[comp * i], r = ref[i][0];
                gmax = std::max(gmax, g);
                if (r > 0.0) ++active;
                dp = std::max(dp, std::abs(g - r) / std::max(pmax, 1e-300));
            }
            dp_all = std::max(dp_all, dp);
            char buf[200];
            std::snprintf(buf, sizeof(buf), "%s{\"ts\": %zu, \"nip\": %ld, \"active\": %ld, \"pmax_ref\": %.9g, \"pmax_gpu\": %.9g, \"dp\": %.3g}",
                          ts ? ", " : "", ts, (long)(n / comp), (long)active, pmax, gmax, dp);
            itf += buf;
        }
        itf += "]";
        // ---- the same problem on two ranks (in-process transport), against a single-rank run with
        // the same options; the V-cycle's exact-solve level is pinned (the reference's level 0): its
        // automatic choice depends on how many subdomains a rank batches (oracle/ref_ranks.hpp).
        // First variant only.
        // Several owner strings (comma-separated): one comparison each, as {"owners": {...}, ...}.
        std::string ranks2 = "null";
        if (argc > 6 && vi == 0) {
            const std::string all = argv[6];
            const bool many = all.find(',') != std::string::npos;
            std::string acc = "{";
            size_t a0 = 0;
            while (a0 <= all.size()) {
                const size_t b0 = std::min(all.find(',', a0), all.size());
                const std::string own = all.substr(a0, b0 - a0);
                a0 = b0 + 1;
                if (own.empty()) continue;
                if (own.size() != c.multGrid.size()) {
                    std::fprintf(stderr, "owners: one digit per subdomain\n");
                    return 2;
                }
                std::vector<int32_t> ow(own.size());
                int nr = 1;
                for (size_t tv = 0; tv < own.size(); ++tv) nr = std::max(nr, (ow[tv] = own[tv] - '0') + 1);
                std::vector<std::array<long, 2>> body;
                for (size_t ts = 0; ts < c.searCont.size(); ++ts) body.push_back({(long)c.contBody[ts][0], (long)c.contBody[ts][1]});
                mgpis_options_t o;
                mgpis_default_options(&o);
                o.coarse_level = 0;
                const std::string r = ddpca_ranks::compare(p, ow, nr, (int64_t)c.multGrid.size(), (int64_t)c.searCont.size(), body, &o);
                if (!many) {
                    ranks2 = r;
                    break;
                }
                acc += (acc.size() > 1 ? ", \"" : "\"") + own + "\": " + r;
            }
            if (many) ranks2 = acc + "}";
        }
        mcontact_gpu_destroy(h);
        ddpca_problem_destroy(p);
        std::fprintf(stderr,
                     "{\"variant\": \"%s\", \"native\": %s, \"K_rel\": %.3g, \"subdomains\": %zu, \"nodes\": %ld, \"hanging_nodes\": %ld, "
                     "\"iters_gpu\": %ld, \"iters_ref\": %ld, "
                     "\"resuDisp_rel\": %.3g, \"moni_rows\": %ld, \"moni_rel\": %.3g, \"pressure_rel\": %.3g, \"interfaces\": %s, "
                     "\"ranks2\": %s, \"multicolour\": %s, \"gs_rows\": [%ld, %ld, %ld]}\n",
                     variants[vi].c_str(), native ? "true" : "false", dK, c.multGrid.size(), nnodes, nhang, (long)n_gpu,
                     (long)c.iterNumbReco, du, (long)kmax, dmoni, dp_all, itf.c_str(), ranks2.c_str(), mcol ? "true" : "false",
                     (long)gsr[0], (long)gsr[1], (long)gsr[2]);
    }
    return 0;
}
