// ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.
//
// LAGRANGE against the reference: the reference builds its own BLOCK example (examples/BLOCK.h,
// domaNumb {1,1,1}: three stacked blocks + six load/support plates, 8 interfaces, glued and
// contact) with an optional tangential component in the top load and Coulomb friction on the
// contact interfaces, runs its own MCONTACT::LAGRANGE(precType) (dual mortar, semi-smooth Newton,
// MGPIS-BiCGSTAB), and the same MULTIGRID hierarchies and integration points then go through
// libddpca_amd's ddpca_lagrange_* (host assembly + device BiCGSTAB).  Compared: the Newton step
// count, the final active set and multipliers (the reference's resuLagr_<ts>.txt), and the
// displacements (reference resuDisp vs OUTP_SUB1 of the device's condensed solution).  One JSON
// line on stderr.
// Record / replay of the reference's answers (so the GPU box need not re-run the reference's
// single-threaded Newton loop each time): DDPCA_REF_RECORD=<dir> writes the reference's progress
// log, its resuLagr_<ts>.txt and resuDisp (raw fp64 per subdomain) there after its LAGRANGE;
// DDPCA_REF_REPLAY=<dir> (when <dir>/log.txt exists) builds the same problem -- MESH, the contact
// searches, then exactly LAGRANGE's own setup (TRANSFER, STIF_MATR, CONSTRAINT(precType == 1 ? 1
// : -1), MCONTACT.h:2847-2860) -- and compares against the recorded answers instead
// (tests/golden/lagrange/*, made by tests/golden/make_lagrange_golden.sh).
//   ref_lagrange globLeve precType fric tangential_load
#include <execinfo.h>
#include <unistd.h>

#include <cmath>
#include <csignal>
#include <cstdio>
#include <fstream>
#include <sstream>

#include <memory>

#include "examples/BLOCK.h"
#include "examples/CYLINDER_1.h"
#include "ref_bind.hpp"

namespace {

struct RefLagr {
    std::vector<long> node, stat;
    std::vector<double> v0, v1, v2;
};

RefLagr read_lagr(const std::string& path) {
    RefLagr r;
    std::ifstream f(path);
    std::string line;
    while (std::getline(f, line)) {
        std::istringstream is(line);
        long n, s;
        double a, b, c;
        if (!(is >> n >> s >> a >> b >> c)) continue;
        r.node.push_back(n);
        r.stat.push_back(s);
        r.v0.push_back(a);
        r.v1.push_back(b);
        r.v2.push_back(c);
    }
    return r;
}

}  // namespace

void on_fault(int sig) {  // a crash names its frames (no debugger on the GPU box)
    void* fr[64];
    const int n = backtrace(fr, 64);
    backtrace_symbols_fd(fr, n, 2);
    std::signal(sig, SIG_DFL);
    std::raise(sig);
}

int main(int argc, char** argv) {
    std::signal(SIGSEGV, on_fault);
    std::signal(SIGABRT, on_fault);
    // ref_lagrange [cylinder] globLeve precType fric tangential_load
    const bool cyl = argc > 1 && std::string(argv[1]) == "cylinder";
    const int a0 = cyl ? 2 : 1;
    const long gl = argc > a0 ? std::atol(argv[a0]) : 1;
    const long prec = argc > a0 + 1 ? std::atol(argv[a0 + 1]) : 1;
    const double fric = argc > a0 + 2 ? std::atof(argv[a0 + 2]) : 0.0;
    const double tang = argc > a0 + 3 ? std::atof(argv[a0 + 3]) : 0.0;
    std::unique_ptr<BLOCK> blk;
    std::unique_ptr<CYLINDER_1> cy;
    if (cyl) cy = std::make_unique<CYLINDER_1>();  // creates ./Cylinder/
    else blk = std::make_unique<BLOCK>();           // creates ./Block/
    MCONTACT& b = cyl ? static_cast<MCONTACT&>(*cy) : static_cast<MCONTACT&>(*blk);
    const std::string outdir = cyl ? "Cylinder" : "Block";
    std::string log = outdir + "/ref_lagrange_stdout.txt";
    const char* rec = std::getenv("DDPCA_REF_RECORD");
    const char* rep = std::getenv("DDPCA_REF_REPLAY");
    const bool replay = rep && std::ifstream(std::string(rep) + "/log.txt").good();
    const int saved = dup(1);
    if (!std::freopen(replay ? "/dev/null" : log.c_str(), "w", stdout)) return 2;  // the reference's progress output, parsed below
    // replay: LAGRANGE's own setup instead of the reference's Newton loop (MCONTACT.h:2847-2860)
    auto lagrange_setup = [&] {
        for (auto& g : b.multGrid) g.leveNode.clear();  // (TRANSFER appends to leveNode)
#pragma omp parallel for
        for (long tv = 0; tv < (long)b.multGrid.size(); ++tv) {
            b.multGrid[tv].TRANSFER();
            b.multGrid[tv].STIF_MATR();
            b.multGrid[tv].CONSTRAINT(prec == 1 ? 1 : -1);
        }
    };
    if (cyl) {
        // CYLINDER_1 (locally refined: hanging non-mortar nodes are dropped, MCONTACT.h:2870-2893),
        // reduced locaLeve as in ref_cylinder; frictionless as the example sets it
        cy->copyNumb = 1;
        cy->locaLeve = 3 + gl;
        cy->globInho = 2;
        cy->bandWidt = 2.0e-4;
        if (replay) {
            cy->SOLVE(0);  // MESH, contact searches, ESTABLISH
            lagrange_setup();
        } else {
            cy->SOLVE(1 + prec);
        }
    } else {
        blk->domaNumb = {1, 1, 1};
        blk->globLeve = gl;
        blk->muscSett = 0;  // no coarse space: ESTABLISH stays cheap and APPS returns at once
        blk->doleMcsc.assign(3 * 1 + 6, 1);
        blk->loadPres << tang, 0.0, -1.0E7;
        blk->ESTA_SURF();
        if (fric == 0.0 && tang == 0.0 && !replay) {
            blk->SOLVE(1 + prec);  // MESH, contact searches, the reference's LAGRANGE(prec)
        } else {
            blk->SOLVE(0);  // MESH, contact searches, ESTABLISH
            for (size_t ts = 0; ts < b.fricCoef.size(); ++ts)
                if (b.fricCoef[ts] == 0.0) b.fricCoef[ts] = fric;  // the contact (not glued) interfaces
            // LAGRANGE re-runs TRANSFER, which appends to leveNode (MULTIGRID.h:884-900): start it
            // from the state MESH left, as SOLVE(2) does
            if (replay) {
                lagrange_setup();
            } else {
                for (auto& g : b.multGrid) g.leveNode.clear();
                b.LAGRANGE(prec);
            }
        }
    }
    std::fflush(stdout);
    dup2(saved, 1);
    auto lagr_file = [&](int64_t ts) {
        return replay ? std::string(rep) + "/resuLagr_" + std::to_string(ts) + ".txt"
                      : DIRECTORY("resuLagr_" + std::to_string(ts) + ".txt");
    };
    if (replay) {
        log = std::string(rep) + "/log.txt";
        b.resuDisp.resize(b.multGrid.size());
        for (size_t tv = 0; tv < b.multGrid.size(); ++tv) {
            // the recorded answer must exist and fit this subdomain's mesh (3 per node), else the
            // comparison below would subtract vectors of different sizes
            const std::string path = std::string(rep) + "/resuDisp_" + std::to_string(tv) + ".bin";
            std::ifstream f(path, std::ios::binary);
            if (!f) {
                std::fprintf(stderr, "replay: cannot open %s\n", path.c_str());
                return 2;
            }
            f.seekg(0, std::ios::end);
            const std::streamoff bytes = f.tellg();
            const std::streamoff n = bytes / (std::streamoff)sizeof(double);
            const std::streamoff want = 3 * (std::streamoff)b.multGrid[tv].nodeCoor.size();
            if (bytes < 0 || n != want || n * (std::streamoff)sizeof(double) != bytes) {
                std::fprintf(stderr, "replay: %s holds %ld doubles, subdomain %zu has %ld dofs\n", path.c_str(), (long)n, tv,
                             (long)want);
                return 2;
            }
            f.seekg(0);
            b.resuDisp[tv].resize(n);
            if (!f.read(reinterpret_cast<char*>(b.resuDisp[tv].data()), n * sizeof(double))) {
                std::fprintf(stderr, "replay: short read of %s\n", path.c_str());
                return 2;
            }
        }
    } else if (rec) {
        const std::string d(rec);
        std::ofstream(d + "/log.txt") << std::ifstream(log).rdbuf();
        for (size_t ts = 0; ts < b.searCont.size(); ++ts)
            std::ofstream(d + "/resuLagr_" + std::to_string(ts) + ".txt") << std::ifstream(lagr_file((int64_t)ts)).rdbuf();
        for (size_t tv = 0; tv < b.resuDisp.size(); ++tv)
            std::ofstream(d + "/resuDisp_" + std::to_string(tv) + ".bin", std::ios::binary)
                .write(reinterpret_cast<const char*>(b.resuDisp[tv].data()), b.resuDisp[tv].size() * sizeof(double));
        std::fprintf(stderr, "recorded the reference's answers in %s\n", rec);
    }
    // the reference's Newton count and BiCGSTAB iterations from its progress output
    long tc_ref = -1;
    std::vector<long> its_ref;
    {
        std::ifstream f(log);
        std::string line;
        long last = -1;
        while (std::getline(f, line)) {
            if (line.rfind("#Iteration: ", 0) == 0) last = std::atol(line.c_str() + 12);
            if (line.rfind("#Iterations: ", 0) == 0) last = std::atol(line.c_str() + 13);  // Eigen::BiCGSTAB
            if (line.find("MGPIS::BiCGSTAB_SOLV") != std::string::npos || line.find("Eigen::BiCGSTAB") != std::string::npos) {
                if (last >= 0) its_ref.push_back(last);
                last = -1;
            }
            const auto p = line.find("Converge after ");
            if (p != std::string::npos) tc_ref = std::atol(line.c_str() + p + 15);
            if (line.find("Converge after") != std::string::npos || line.find("unconverged constraints") != std::string::npos) {
                if (last >= 0) its_ref.push_back(last);
                last = -1;
            }
        }
    }
    // the same problem through the C ABI
    const int64_t nsub = (int64_t)b.multGrid.size(), nint = (int64_t)b.searCont.size();
    ddpca_lagrange_t h = nullptr;
    ddpca_bind::check(ddpca_lagrange_create(nsub, nint, &h));
    for (int64_t tv = 0; tv < nsub; ++tv) {
        MULTIGRID& g = b.multGrid[tv];
        const long L = g.mgpi.maxiLeve;
        // precType 2 runs CONSTRAINT(-1): no MGPIS hierarchy, only the fine level (MCONTACT.h:2854-2859)
        std::vector<ddpca_bind::Csr> K, P;
        std::vector<int64_t> nnodes, nfree;
        std::vector<std::vector<int32_t>> fd;
        std::vector<const int32_t*> fdp;
        int64_t acc = 0;
        for (long l = 0; l <= L; ++l) {
            acc += (int64_t)g.leveNode[l].size();
            if (prec == 2 && l < L) continue;
            ddpca_bind::SpMat C = g.consOper[l];
            C.makeCompressed();
            fd.emplace_back(C.innerIndexPtr(), C.innerIndexPtr() + C.rows());
            nnodes.push_back(acc);
            nfree.push_back(C.rows());
            K.emplace_back(g.mgpi.consStif[l]);
            if (l < L) P.emplace_back(g.mgpi.realProl[l]);
        }
        for (auto& f : fd) fdp.push_back(f.data());
        const ddpca_bind::Csr G(ddpca_bind::SpMat(g.earlTran * g.prolOper[L] * ddpca_bind::SpMat(g.consOper[L].transpose())));
        std::vector<ddpca_csr_t> Kv, Pv;
        for (auto& k : K) Kv.push_back(k.view());
        for (auto& q : P) Pv.push_back(q.view());
        const int64_t nall = (int64_t)g.nodeCoor.size();
        std::vector<uint8_t> hang(nall, 0);
        for (int64_t n = 0; n < nall; ++n)
            if (g.nodeLepo[n][0] == L + 1) hang[n] = 1;
        const ddpca_csr_t gv = G.view();
        ddpca_bind::check(ddpca_lagrange_set_subdomain(h, tv, (int)K.size(), nnodes.data(), nfree.data(), fdp.data(), Kv.data(),
                                                       Pv.data(), g.consForc.data(), nall, &gv, hang.data()));
    }
    for (int64_t ts = 0; ts < nint; ++ts) {
        const auto& ips = b.searCont[ts].intePoin;
        const int64_t n = (int64_t)ips.size();
        std::vector<int64_t> node(8 * n);
        std::vector<double> shap(8 * n), basis(9 * n), gap(n), w(n);
        for (int64_t i = 0; i < n; ++i) {
            for (int s = 0; s < 2; ++s)
                for (int k = 0; k < 4; ++k) {
                    node[8 * i + 4 * s + k] = ips[i].node[s][k];
                    shap[8 * i + 4 * s + k] = ips[i].shapFunc[s][k];
                }
            for (int a = 0; a < 3; ++a)
                for (int c = 0; c < 3; ++c) basis[9 * i + 3 * a + c] = ips[i].basiVect[a](c);
            gap[i] = ips[i].initNgap;
            w[i] = ips[i].quadWeig;
        }
        ddpca_bind::check(ddpca_lagrange_set_interface(h, ts, b.contBody[ts][0], b.contBody[ts][1], b.fricCoef[ts], n, node.data(),
                                                       shap.data(), basis.data(), gap.data(), w.data()));
    }
    const int64_t tc = ddpca_lagrange_solve(h, 0, (int)prec, nullptr, 50);
    ddpca_bind::check((int)std::min<int64_t>(tc, 0));
    std::vector<double> its(64);
    const int64_t nst = ddpca_lagrange_get(h, "solver_iters", 0, its.data(), (int64_t)its.size());
    std::vector<double> rel(64), brk(64);
    ddpca_lagrange_get(h, "solver_relres", 0, rel.data(), (int64_t)rel.size());
    ddpca_lagrange_get(h, "solver_breakdown", 0, brk.data(), (int64_t)brk.size());
    std::vector<double> cinv(3 * nst);
    ddpca_lagrange_get(h, "coarse_inverse", 0, cinv.data(), (int64_t)cinv.size());
    // displacements: OUTP_SUB1 of the device's condensed solution vs the reference's resuDisp
    double du = 0.0;
    for (int64_t tv = 0; tv < nsub; ++tv) {
        MULTIGRID& g = b.multGrid[tv];
        Eigen::VectorXd u(g.mgpi.consStif[g.mgpi.maxiLeve].rows());
        ddpca_bind::check((int)std::min<int64_t>(ddpca_lagrange_get(h, "u", tv, u.data(), u.size()), 0));
        Eigen::VectorXd disp;
        g.OUTP_SUB1(u, disp);
        du = std::max(du, (disp - b.resuDisp[tv]).norm() / std::max(b.resuDisp[tv].norm(), 1e-300));
    }
    // multipliers and active sets vs resuLagr_<ts>.txt
    std::string itf = "[";
    bool nodes_equal = true, stat_equal = true;
    double dl = 0.0;
    for (int64_t ts = 0; ts < nint; ++ts) {
        const RefLagr r = read_lagr(lagr_file(ts));
        const int64_t m = ddpca_lagrange_get(h, "node", ts, nullptr, 0);
        std::vector<double> nd(m), st(m), lam(3 * m);
        ddpca_lagrange_get(h, "node", ts, nd.data(), m);
        ddpca_lagrange_get(h, "status", ts, st.data(), m);
        ddpca_lagrange_get(h, "lambda", ts, lam.data(), 3 * m);
        bool ne = (int64_t)r.node.size() == m, se = true;
        double scale = 0.0, d = 0.0;
        int nstat[3] = {0, 0, 0};
        for (int64_t i = 0; i < std::min<int64_t>(m, (int64_t)r.node.size()); ++i) {
            ne = ne && (long)nd[i] == r.node[i];
            se = se && (long)st[i] == r.stat[i];
            if (st[i] >= 0 && st[i] <= 2) nstat[(int)st[i]]++;
            // the file holds lambda_n, then (lambda_t1, lambda_t2), or (mu lambda_n, 0) on sliding nodes
            const double t1 = r.stat[i] == 1 ? b.fricCoef[ts] * lam[3 * i] : lam[3 * i + 1];
            const double t2 = r.stat[i] == 1 ? 0.0 : lam[3 * i + 2];
            scale = std::max({scale, std::abs(r.v0[i]), std::abs(r.v1[i]), std::abs(r.v2[i])});
            d = std::max({d, std::abs(lam[3 * i] - r.v0[i]), std::abs(t1 - r.v1[i]), std::abs(t2 - r.v2[i])});
        }
        const double rel = scale > 0 ? d / scale : d;
        dl = std::max(dl, rel);
        nodes_equal = nodes_equal && ne;
        stat_equal = stat_equal && se;
        char buf[240];
        std::snprintf(buf, sizeof(buf), "%s{\"ts\": %ld, \"fric\": %g, \"nodes\": %ld, \"open\": %d, \"slip\": %d, \"stick\": %d, \"lambda_rel\": %.3g, \"lambda_max\": %.6g}",
                      ts ? ", " : "", (long)ts, b.fricCoef[ts], (long)m, nstat[0], nstat[1], nstat[2], rel, scale);
        itf += buf;
    }
    itf += "]";
    std::string sit = "[", rit = "[", srel = "[", sbrk = "[", scin = "[";
    for (int64_t k = 0; k < nst; ++k) {
        char nb[32], cb[96];
        std::snprintf(cb, sizeof(cb), "%s[%d, %.3e, %ld]", k ? ", " : "", (int)cinv[3 * k],
                      std::isfinite(cinv[3 * k + 1]) ? cinv[3 * k + 1] : -1.0, (long)cinv[3 * k + 2]);
        scin += cb;
        std::snprintf(nb, sizeof(nb), "%.3e", rel[k]);
        sit += (k ? ", " : "") + std::to_string((long)its[k]);
        srel += (k ? ", " : "") + std::string(nb);
        sbrk += (k ? ", " : "") + std::to_string((int)brk[k]);
    }
    srel += "]";
    sbrk += "]";
    scin += "]";
    for (size_t k = 0; k < its_ref.size(); ++k) rit += (k ? ", " : "") + std::to_string(its_ref[k]);
    sit += "]";
    rit += "]";
    ddpca_lagrange_destroy(h);
    std::fprintf(stderr,
                 "{\"newton\": %ld, \"newton_ref\": %ld, \"bicgstab_iters\": %s, \"bicgstab_iters_ref\": %s, "
                 "\"bicgstab_relres\": %s, \"bicgstab_breakdown\": %s, \"coarse_inverse\": %s, \"resuDisp_rel\": %.3g, "
                 "\"lambda_rel\": %.3g, \"nodes_equal\": %s, \"status_equal\": %s, \"replayed\": %s, \"interfaces\": %s}\n",
                 (long)tc, tc_ref, sit.c_str(), rit.c_str(), srel.c_str(), sbrk.c_str(), scin.c_str(), du, dl, nodes_equal ? "true" : "false", stat_equal ? "true" : "false",
                 replay ? "true" : "false", itf.c_str());
    return 0;
}
