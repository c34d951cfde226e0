// ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.
//
// The reference's OWN ADMM iteration timed on the bench's workload (bench.py `cpu_baseline`,
// profiles/ref_admm_time.py): the reference's MCONTACT (MCONTACT.h:9-95) is filled from a
// directory of raw operators written by the device run at its final state, and its unmodified
// MCONTACT::CONTACT_ANALYSIS (MCONTACT.h:2493-2723) runs -- the body balance with every
// subdomain's MGPIS::CG_SOLV(1) in its omp parallel for (2511-2537), the interface-eliminated
// coarse correction with its SimplicialLDLT coarse solve (2578-2612), the interface step with the
// LDLT-factorised surface mass matrices (2629-2704), MONITOR (2725-2845) and the per-iteration text
// output (OUTP_SUB2, OUTPUT_PRTR, resuMoni.txt) into a scratch directory, as the reference does.
// Its stdout is read by a watcher thread that timestamps the "The <tc>-th iteration" lines; once
// iteration `stop` starts, the per-iteration wall times are printed as one JSON line on stderr and
// the process ends (CONTACT_ANALYSIS has no iteration cap below 3000).  Nothing is computed here:
// the harness only assigns the reference's public members.
//
//   ref_admm_time DIR OUTDIR STOP
//
// DIR/meta.txt lines: "nsub N", "nint M", "muscSett m", "sub tv N nlev nfree", "csr NAME rows cols nnz",
// "vec NAME n", "ivec NAME n", "iface ts body0 body1 fric nip"; arrays NAME.ptr (int64), NAME.col
// (int32), NAME.val (float64), NAME.f64, NAME.i64.  Names: K<tv>_<l>, P<tv>_<l>, consFlag<tv>,
// consForc<tv>, cdof<tv> / cval<tv> (consDofv), u<tv>, for interface ts and side s systTran<ts>_<s>,
// systTran_pena, inteMass, inteMass_pena, inpoLagr, pemaInpo_r, inteInpo, aux<ts>_<s>,
// lam<ts>_<s>, pemaDiag<ts>, inpoNgap<ts>, basis<ts> (9 per ip); coarse: globCoup_1,
// globTran_1<ts>_<s>, globTran_D_1<tv>, globForc_1, accuProl<tv>, baseReco, doleMcsc.
#include "MCONTACT.h"

#include <omp.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <fstream>
#include <map>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

namespace {

using SpMat = Eigen::SparseMatrix<double, Eigen::RowMajor>;

struct Meta {
    std::map<std::string, std::vector<long>> csr;  // rows cols nnz
    std::map<std::string, long> vec, ivec;
    std::map<std::string, long> scal;
    std::vector<std::vector<long>> subs;           // tv N nlev nfree
    std::vector<std::vector<double>> ifaces;       // ts b0 b1 fric nip
};

template <typename T>
std::vector<T> read_raw(const std::string& path, long n) {
    std::vector<T> v(n);
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open " + path);
    f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)(n * sizeof(T)));
    if (!f) throw std::runtime_error("short read " + path);
    return v;
}

std::string g_dir;
Meta g_meta;

SpMat csr(const std::string& name) {
    auto it = g_meta.csr.find(name);
    if (it == g_meta.csr.end()) throw std::runtime_error("missing csr " + name);
    const long r = it->second[0], c = it->second[1], z = it->second[2];
    const auto ptr = read_raw<int64_t>(g_dir + "/" + name + ".ptr", r + 1);
    const auto col = read_raw<int32_t>(g_dir + "/" + name + ".col", z);
    const auto val = read_raw<double>(g_dir + "/" + name + ".val", z);
    std::vector<Eigen::Triplet<double>> t;
    t.reserve(z);
    for (long i = 0; i < r; ++i)
        for (int64_t k = ptr[i]; k < ptr[i + 1]; ++k) t.emplace_back(i, col[k], val[k]);
    SpMat m(r, c);
    m.setFromTriplets(t.begin(), t.end());
    m.makeCompressed();
    return m;
}

Eigen::VectorXd vec(const std::string& name) {
    const long n = g_meta.vec.at(name);
    const auto v = read_raw<double>(g_dir + "/" + name + ".f64", n);
    return Eigen::Map<const Eigen::VectorXd>(v.data(), n);
}

std::vector<int64_t> ivec(const std::string& name) { return read_raw<int64_t>(g_dir + "/" + name + ".i64", g_meta.ivec.at(name)); }

void read_meta() {
    std::ifstream f(g_dir + "/meta.txt");
    if (!f) throw std::runtime_error("meta.txt");
    std::string line;
    while (std::getline(f, line)) {
        std::istringstream s(line);
        std::string kind, name;
        s >> kind;
        if (kind == "csr") {
            long r, c, z;
            s >> name >> r >> c >> z;
            g_meta.csr[name] = {r, c, z};
        } else if (kind == "vec") {
            long n;
            s >> name >> n;
            g_meta.vec[name] = n;
        } else if (kind == "ivec") {
            long n;
            s >> name >> n;
            g_meta.ivec[name] = n;
        } else if (kind == "sub") {
            std::vector<long> v(4);
            for (auto& x : v) s >> x;
            g_meta.subs.push_back(v);
        } else if (kind == "iface") {
            std::vector<double> v(5);
            for (auto& x : v) s >> x;
            g_meta.ifaces.push_back(v);
        } else if (!kind.empty()) {
            long v;
            s >> v;
            g_meta.scal[kind] = v;
        }
    }
}

// progress on stderr (a long run must show it is alive; stdout belongs to the reference)
void progress(const std::string& what, std::chrono::steady_clock::time_point t0) {
    std::fprintf(stderr, "[ref_admm_time] %s (%.1f s)\n", what.c_str(),
                 std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
    std::fflush(stderr);
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: ref_admm_time DIR OUTDIR STOP\n");
        return 2;
    }
    g_dir = argv[1];
    outpDire = std::string(argv[2]) + "/";
    const long stop = std::atol(argv[3]);
    const auto t_setup = std::chrono::steady_clock::now();
    read_meta();
    const long nsub = g_meta.scal.at("nsub"), nint = g_meta.scal.at("nint");
    if (nsub > MAXI_DOMA_NUMB || nint > MAXI_INTE_NUMB) throw std::runtime_error("too many subdomains / interfaces");
    auto* mc = new MCONTACT();
    mc->muscSett = g_meta.scal.at("muscSett");
    mc->multGrid.resize(nsub);
    mc->resuDisp.resize(nsub);
    // ---- subdomains: the MULTIGRID members the ADMM loop reads (ADDITIONAL_FORCE, OUTP_SUB1/2,
    //      MGPIS::CG_SOLV); node numbering = positions (the workload's uniform boxes have no hanging
    //      level: earlTran = prolOper[maxiLeve] = I)
    for (long i = 0; i < nsub; ++i) {
        const auto& sd = g_meta.subs[i];
        const long tv = sd[0], N = sd[1], nlev = sd[2], nfree = sd[3];
        MULTIGRID& g = mc->multGrid[tv];
        g.mgpi.maxiLeve = nlev - 1;
        for (long l = 0; l < nlev; ++l) g.mgpi.consStif.push_back(csr("K" + std::to_string(tv) + "_" + std::to_string(l)));
        for (long l = 0; l + 1 < nlev; ++l) g.mgpi.realProl.push_back(csr("P" + std::to_string(tv) + "_" + std::to_string(l)));
        for (long n = 0; n < N; ++n) g.nodeCoor[n] = COOR();
        g.nodeLepo.assign(N, std::vector<long>{0, 0});
        for (long n = 0; n < N; ++n) g.nodeLepo[n][1] = n;
        SpMat I(3 * N, 3 * N);
        I.setIdentity();
        g.earlTran = I;
        g.prolOper.assign(nlev, SpMat());
        g.prolOper[nlev - 1] = I;
        g.origStif.assign(nlev, SpMat());
        g.origStif[nlev - 1].resize(3 * N, 3 * N);
        const auto flag = ivec("consFlag" + std::to_string(tv));
        g.consFlag.resize(3 * N);
        std::vector<Eigen::Triplet<double>> t;
        for (long d = 0, k = 0; d < 3 * N; ++d) {
            g.consFlag(d) = (int)flag[d];
            if (flag[d]) t.emplace_back(k++, d, 1.0);
        }
        g.consOper.assign(nlev, SpMat());
        g.consOper[nlev - 1].resize(nfree, 3 * N);
        g.consOper[nlev - 1].setFromTriplets(t.begin(), t.end());
        g.consForc = vec("consForc" + std::to_string(tv));
        if (g_meta.ivec.count("cdof" + std::to_string(tv))) {
            const auto cd = ivec("cdof" + std::to_string(tv));
            const Eigen::VectorXd cv = vec("cval" + std::to_string(tv));
            for (size_t k = 0; k < cd.size(); ++k) g.consDofv[cd[k]] = cv((long)k);
        }
        mc->resuDisp[tv] = vec("u" + std::to_string(tv));
        progress("subdomain " + std::to_string(tv) + " read", t_setup);
    }
    // ---- interfaces (MCONTACT::ESTABLISH's outputs)
    mc->searCont.resize(nint);
    mc->contBody.assign(nint, std::vector<long>(2));
    mc->fricCoef.assign(nint, 0.0);
    for (auto* S : {&mc->systTran, &mc->systTran_pena, &mc->inteMass, &mc->inteMass_pena, &mc->inpoLagr, &mc->inteInpo})
        S->assign(nint, std::vector<SpMat>(2));
    mc->pemaInpo_r.assign(nint, std::vector<SpMat>(2));
    mc->pemaInpo.assign(nint, SpMat());
    mc->inpoNgap.assign(nint, Eigen::VectorXd());
    mc->inteAuxi.assign(nint, std::vector<Eigen::VectorXd>(2));
    mc->inteLagr.assign(nint, std::vector<Eigen::VectorXd>(2));
    for (const auto& it : g_meta.ifaces) {
        const long ts = (long)it[0];
        mc->contBody[ts] = {(long)it[1], (long)it[2]};
        mc->fricCoef[ts] = it[3];
        const long nip = (long)it[4];
        const std::string T = std::to_string(ts);
        const Eigen::VectorXd basis = vec("basis" + T);
        mc->searCont[ts].intePoin.resize(nip);
        for (long q = 0; q < nip; ++q)
            for (int a = 0; a < 3; ++a)
                mc->searCont[ts].intePoin[q].basiVect[a] << basis(9 * q + 3 * a), basis(9 * q + 3 * a + 1), basis(9 * q + 3 * a + 2);
        for (int s = 0; s < 2; ++s) {
            const std::string S = T + "_" + std::to_string(s);
            mc->systTran[ts][s] = csr("systTran" + S);
            mc->systTran_pena[ts][s] = csr("systTran_pena" + S);
            mc->inteMass[ts][s] = csr("inteMass" + S);
            mc->inteMass_pena[ts][s] = csr("inteMass_pena" + S);
            mc->inpoLagr[ts][s] = csr("inpoLagr" + S);
            mc->pemaInpo_r[ts][s] = csr("pemaInpo_r" + S);
            mc->inteInpo[ts][s] = csr("inteInpo" + S);
            mc->inteAuxi[ts][s] = vec("aux" + S);
            mc->inteLagr[ts][s] = vec("lam" + S);
        }
        const Eigen::VectorXd pd = vec("pemaDiag" + T);
        SpMat D(pd.size(), pd.size());
        std::vector<Eigen::Triplet<double>> t;
        for (long k = 0; k < pd.size(); ++k) t.emplace_back(k, k, pd(k));
        D.setFromTriplets(t.begin(), t.end());
        mc->pemaInpo[ts] = D;
        mc->inpoNgap[ts] = vec("inpoNgap" + T);
        progress("interface " + T + " read", t_setup);
    }
    // ---- interface-eliminated coarse space (MULTISCALE_1's outputs)
    if ((mc->muscSett >> 1) % 2 == 1) {
        mc->globCoup_1 = csr("globCoup_1");
        mc->globForc_1 = vec("globForc_1");
        mc->globTran_1.assign(nint, std::vector<SpMat>(2));
        for (long ts = 0; ts < nint; ++ts)
            for (int s = 0; s < 2; ++s) mc->globTran_1[ts][s] = csr("globTran_1" + std::to_string(ts) + "_" + std::to_string(s));
        mc->globTran_D_1.resize(nsub);
        mc->accuProl.resize(nsub);
        for (long tv = 0; tv < nsub; ++tv) {
            mc->globTran_D_1[tv] = csr("globTran_D_1" + std::to_string(tv));
            mc->accuProl[tv] = csr("accuProl" + std::to_string(tv));
        }
        const auto br = ivec("baseReco"), dm = ivec("doleMcsc");
        mc->baseReco.assign(br.begin(), br.end());
        mc->doleMcsc.assign(dm.begin(), dm.end());
    }
    // ---- the reference's own setup steps (MCONTACT::ESTABLISH 828-847, MULTISCALE_1 1857-1865):
    //      MGPIS::ESTABLISH per subdomain, the LDLT factorisations -- untimed
#pragma omp parallel for schedule(dynamic, 1)
    for (long tv = 0; tv < nsub; ++tv) {
        MULTIGRID& g = mc->multGrid[tv];
        g.mgpi.ESTABLISH();
        // small subdomains take the pre-factorised LDLT instead of CG_SOLV (MCONTACT.h:828-835, 2527)
        if (3 * (long)g.nodeCoor.size() < DIRE_MAXI_SUBD) mc->mugrDiso[tv].compute(g.mgpi.consStif[g.mgpi.maxiLeve]);
    }
#pragma omp parallel for schedule(dynamic, 1)
    for (long k = 0; k < 2 * nint; ++k) {
        const long ts = k / 2, s = k % 2;
        if (mc->inteMass[ts][s].rows() < DIRE_MAXI) mc->inteDiso[ts][s].compute(mc->inteMass[ts][s]);
        if (mc->inteMass_pena[ts][s].rows() < DIRE_MAXI) mc->inteDiso_pena[ts][s].compute(mc->inteMass_pena[ts][s]);
    }
    if ((mc->muscSett >> 1) % 2 == 1 && mc->globCoup_1.rows() < DIRE_MAXI) mc->coarSolv_D_1.compute(mc->globCoup_1);
    progress("setup done (MGPIS::ESTABLISH, LDLT factorisations)", t_setup);
    const double setup_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_setup).count();
    // ---- CONTACT_ANALYSIS with its stdout on a pipe: a watcher timestamps the iteration lines
    int fd[2];
    if (pipe(fd) != 0) throw std::runtime_error("pipe");
    std::fflush(stdout);
    std::cout.flush();
    const int saved = dup(1);
    dup2(fd[1], 1);
    close(fd[1]);
    std::thread watcher([&, saved] {
        FILE* in = fdopen(fd[0], "r");
        char buf[4096];
        std::vector<double> t_start;
        const auto t0 = std::chrono::steady_clock::now();
        while (std::fgets(buf, sizeof(buf), in)) {
            const std::string l(buf);
            const auto p = l.find("-th iteration");
            if (p != std::string::npos && l.rfind("The ", 0) == 0) {
                t_start.push_back(std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
                progress("reference iteration " + std::to_string(t_start.size() - 1) + " starts", t0);
                if ((long)t_start.size() > stop) {
                    std::string its;
                    for (size_t k = 1; k < t_start.size(); ++k)
                        its += (k > 1 ? ", " : "") + std::to_string(t_start[k] - t_start[k - 1]);
                    std::fprintf(stderr,
                                 "{\"iteration_s\": [%s], \"threads\": %d, \"setup_s\": %.3f, \"nsub\": %ld, \"nint\": %ld, "
                                 "\"muscSett\": %ld}\n",
                                 its.c_str(), omp_get_max_threads(), setup_s, nsub, nint, (long)mc->muscSett);
                    std::fflush(stderr);
                    _exit(0);
                }
            }
        }
        (void)saved;
    });
    mc->CONTACT_ANALYSIS();
    std::cout.flush();
    std::fflush(stdout);
    dup2(saved, 1);
    std::fprintf(stderr, "{\"error\": \"CONTACT_ANALYSIS ended before iteration %ld\"}\n", stop);
    _exit(3);
}
