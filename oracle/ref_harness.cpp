// ORACLE TEST INFRASTRUCTURE -- NOT PART OF THE PRODUCT.
//
// Drives the reference implementation (QuanchengP/DDPCA-ADMM, header-only C++17, compiled in
// place from /root/reference by oracle/Makefile into oracle/_ref/) to produce golden fixtures
// for the hot path: MGPIS::CG_SOLV / MULT_VCYC (MGPIS.h:55-225), the MULTIGRID operator
// pipeline (MULTIGRID.h:756-1255) and MCONTACT::CONTACT_ANALYSIS (MCONTACT.h:2493-2845).
// Nothing in here is shipped or linked into ddpca-admm_amd; only tests/ and bench.py's
// cpu_baseline leg may run it.  No reference source is copied: this file only #includes the
// reference headers where they lie and calls their public members.
//
// Modes (outputs are .npy files in <outdir>, plus the reference's own text outputs in CWD):
//   beam_nodd d0 d1 d2 globLeve outdir full(0/1) [cg(0/1)]
//       single-domain BEAM (BEAM.h:251-311, 403-422) -> level fingerprints, consForc,
//       one V-cycle application, CG_SOLV(1) and CG_SOLV(0) solutions + iteration counts.
//   beam_dd d0 d1 d2 globLeve D0 D1 D2 outdir [muscSett]
//       DD BEAM with glued interfaces (fricCoef=-1, BEAM.h:424-610), muscSett = 0 unless given.
//   twoblock fric globLeve outdir [muscSett]
//       two stacked blocks, one contact interface (fric = 0: frictionless, > 0: Coulomb),
//       built from the reference's MULTIGRID/CSEARCH/CURVEDS/MCONTACT API.
//   With muscSett = 2 (interface-eliminated coarse space, MCONTACT.h:1672-2301) doleMcsc = 1
//   for every subdomain (the examples' setting, e.g. BLOCK.h:38-41, DEHW.h:2222, 2239) and the
//   coarse operators globCoup_1 / globForc_1 / globTran_1 / globTran_D_1 / accuProl are dumped;
//   with muscSett = 1 (LATIN-type, MULTISCALE, MCONTACT.h:898-1536; CYLINDER.h:42) likewise
//   globCoup / globTran / globTran_pena / globTran_D / accuProl.
//   beam_solv d0 d1 d2 globLeve outdir
//       the same BEAM -> MULT_SOLV, BiCGSTAB_SOLV(0/1), GMRES_SOLV(0/1) solutions.
//   time_cg d0 d1 d2 globLeve reps
//       wall time of MGPIS::CG_SOLV(1) on the BEAM mesh (CPU baseline calibration).
//   time_cg_ops dir reps
//       wall time of MGPIS::CG_SOLV(1) on a hierarchy handed over as raw files (bench.py's
//       cpu_baseline: a headline subdomain's consStif[l] / realProl[l] and its right-hand side):
//       dir/meta.txt = "nlev" then "rows cols nnz" per K level and per P level; dir/K<l>.ptr (int64),
//       .col (int32), .val (float64), the same for P<l>, dir/b.f64.
#include "examples/BEAM.h"

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <random>
#include <regex>
#include <stdexcept>
#include <string>

#include <unistd.h>

namespace harness {

// ---------------------------------------------------------------- .npy writer
template <typename T> const char* npy_descr();
template <> const char* npy_descr<double>() { return "<f8"; }
template <> const char* npy_descr<int64_t>() { return "<i8"; }
template <> const char* npy_descr<int32_t>() { return "<i4"; }

template <typename T>
void save_npy(const std::string& path, const T* data, const std::vector<size_t>& shape) {
    std::string dict = "{'descr': '";
    dict += npy_descr<T>();
    dict += "', 'fortran_order': False, 'shape': (";
    size_t count = 1;
    for (size_t i = 0; i < shape.size(); ++i) {
        dict += std::to_string(shape[i]);
        dict += (shape.size() == 1) ? "," : (i + 1 < shape.size() ? ", " : "");
        count *= shape[i];
    }
    dict += "), }";
    size_t hdr = 10 + dict.size() + 1;
    size_t pad = (64 - hdr % 64) % 64;
    dict.append(pad, ' ');
    dict += '\n';
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) { std::perror(path.c_str()); std::exit(2); }
    const unsigned char magic[8] = {0x93, 'N', 'U', 'M', 'P', 'Y', 1, 0};
    std::fwrite(magic, 1, 8, f);
    uint16_t hlen = (uint16_t)dict.size();
    std::fwrite(&hlen, 2, 1, f);
    std::fwrite(dict.data(), 1, dict.size(), f);
    if (count) std::fwrite(data, sizeof(T), count, f);
    std::fclose(f);
}

std::string g_out;
std::string P(const std::string& name) { return g_out + "/" + name + ".npy"; }

void save_vec(const std::string& name, const Eigen::VectorXd& v) {
    save_npy(P(name), v.data(), {(size_t)v.size()});
}
void save_dvec(const std::string& name, const std::vector<double>& v) {
    save_npy(P(name), v.data(), {v.size()});
}
void save_ivec(const std::string& name, const std::vector<int64_t>& v) {
    save_npy(P(name), v.data(), {v.size()});
}
void save_scalar(const std::string& name, double x) { save_npy(P(name), &x, {1}); }

// Full CSR dump of a row-major Eigen sparse matrix: <name>_ptr, _col, _val, _shape.
void save_csr(const std::string& name, Eigen::SparseMatrix<double, Eigen::RowMajor> m) {
    m.makeCompressed();
    std::vector<int64_t> ptr(m.outerIndexPtr(), m.outerIndexPtr() + m.rows() + 1);
    std::vector<int64_t> col(m.innerIndexPtr(), m.innerIndexPtr() + m.nonZeros());
    std::vector<double> val(m.valuePtr(), m.valuePtr() + m.nonZeros());
    save_ivec(name + "_ptr", ptr);
    save_ivec(name + "_col", col);
    save_dvec(name + "_val", val);
    save_ivec(name + "_shape", {(int64_t)m.rows(), (int64_t)m.cols()});
}

// Deterministic probe vector used by every fingerprint: integer arithmetic and one correctly
// rounded division, so every compiler/libm (and numpy) produces the same bits -- a libm sin()
// with FMA-contracted arguments (-march=native) does not.
Eigen::VectorXd probe(long n) {
    Eigen::VectorXd v(n);
    for (long i = 0; i < n; ++i) v(i) = (double)((i * 7919 + 13) % 2003) / 2003.0 - 0.5;
    return v;
}

// Fingerprint of a sparse matrix: [rows, cols, nnz, ||A||_F, sum(A), sum|A|] + A*probe.
void save_fp(const std::string& name, const Eigen::SparseMatrix<double, Eigen::RowMajor>& m) {
    double s = 0, sa = 0;
    for (long r = 0; r < m.outerSize(); ++r)
        for (RSPA_INNE it(m, r); it; ++it) { s += it.value(); sa += std::abs(it.value()); }
    std::vector<double> head = {(double)m.rows(), (double)m.cols(), (double)m.nonZeros(),
                                m.norm(), s, sa};
    save_dvec(name + "_fp", head);
    Eigen::VectorXd y = m * probe(m.cols());
    save_vec(name + "_Kv", y);
}

void save_coords(const std::string& name, const MULTIGRID& g) {
    std::vector<double> c;
    c.reserve(3 * g.nodeCoor.size());
    for (const auto& it : g.nodeCoor) { c.push_back(it.second[0]); c.push_back(it.second[1]); c.push_back(it.second[2]); }
    save_npy(P(name), c.data(), {g.nodeCoor.size(), 3});
}

void save_elems(const std::string& name, const MULTIGRID& g) {
    std::vector<int64_t> e;
    for (const auto& el : g.elemVect)
        if (el.children.empty())
            for (long k = 0; k < 8; ++k) e.push_back(el.cornNode[k]);
    save_npy(P(name), e.data(), {e.size() / 8, 8});
}

// Run fn with the process's stdout captured at the file-descriptor level and return the last
// "#Iteration: N" value + 1 (= loop count of MGPIS::CG_SOLV, which prints iterNumb - 1 at exit,
// MGPIS.h:221).  The reference prints from inside its OpenMP subdomain loop (MCONTACT.h:2511-2537),
// so the capture must be safe under concurrent writers: std::cout stays on its stdio-synchronised
// buffer (stdio locks each call) and fd 1 is pointed at an anonymous temp file for the duration;
// a std::stringbuf swapped into std::cout would be written by several threads unsynchronised.
template <typename F>
long capture_iters(F fn, std::string* text = nullptr) {
    std::cout.flush();
    std::fflush(stdout);
    std::FILE* tmp = std::tmpfile();
    const int saved = dup(1);
    if (!tmp || saved < 0 || dup2(fileno(tmp), 1) < 0) {
        if (tmp) std::fclose(tmp);
        if (saved >= 0) close(saved);
        throw std::runtime_error("capture_iters: cannot redirect stdout");
    }
    try {
        fn();
    } catch (...) {
        std::cout.flush();
        std::fflush(stdout);
        dup2(saved, 1);
        close(saved);
        std::fclose(tmp);
        throw;
    }
    std::cout.flush();
    std::fflush(stdout);
    dup2(saved, 1);
    close(saved);
    std::string s;
    std::rewind(tmp);
    char buf[1 << 16];
    for (size_t k; (k = std::fread(buf, 1, sizeof buf, tmp)) > 0;) s.append(buf, k);
    std::fclose(tmp);
    if (text) *text = s;
    std::regex re("#Iteration: (-?[0-9]+)");
    long last = -2;
    for (std::sregex_iterator it(s.begin(), s.end(), re), end; it != end; ++it)
        last = std::stol((*it)[1]);
    return last + 1;
}

// Silence the reference's progress output around setup calls (same fd-level redirection).
template <typename F>
void quiet(F fn) {
    capture_iters(fn);
}

double now_s() {
    return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Per-level operator dump of one MULTIGRID after CONSTRAINT(1).
void dump_grid(const std::string& pre, MULTIGRID& g, bool full) {
    save_coords(pre + "coords", g);
    save_elems(pre + "elems", g);
    std::vector<int64_t> flag(g.consFlag.data(), g.consFlag.data() + g.consFlag.size());
    save_ivec(pre + "consFlag", flag);
    save_vec(pre + "consForc", g.consForc);
    save_vec(pre + "dispForc", g.dispForc);
    std::vector<int64_t> lev;
    for (long l = 0; l <= g.mgpi.maxiLeve; ++l) lev.push_back(g.mgpi.consStif[l].rows());
    save_ivec(pre + "level_rows", lev);
    std::vector<int64_t> leveN;
    for (const auto& v : g.leveNode) leveN.push_back((int64_t)v.size());
    save_ivec(pre + "level_nodes", leveN);
    std::vector<int64_t> lepo;
    for (const auto& v : g.nodeLepo) { lepo.push_back(v[0]); lepo.push_back(v[1]); }
    save_ivec(pre + "nodeLepo", lepo);
    for (long l = 0; l <= g.mgpi.maxiLeve; ++l) {
        save_fp(pre + "K" + std::to_string(l), g.mgpi.consStif[l]);
        if (full) save_csr(pre + "K" + std::to_string(l), g.mgpi.consStif[l]);
    }
    for (long l = 0; l < g.mgpi.maxiLeve; ++l) {
        save_fp(pre + "P" + std::to_string(l), g.mgpi.realProl[l]);
        if (full) save_csr(pre + "P" + std::to_string(l), g.mgpi.realProl[l]);
    }
}

// ---------------------------------------------------------------- modes
int beam_nodd(long d0, long d1, long d2, long gl, bool full, bool do_cg) {
    BEAM beam(0);
    beam.diviNumb = {d0, d1, d2};
    beam.globLeve = gl;
    quiet([&] { beam.MESH_NODD(0); });
    MULTIGRID& g = beam.multGrid[0];
    double t0 = now_s();
    quiet([&] { g.TRANSFER(); g.STIF_MATR(); g.CONSTRAINT(1); });
    double t_setup = now_s() - t0;
    dump_grid("", g, full);
    const long L = g.mgpi.maxiLeve;
    // One application of the SGS V-cycle preconditioner to consForc (MGPIS.h:55-128).
    {
        DIRE_SOLV ds;
        ds.compute(g.mgpi.consStif[0]);
        Eigen::VectorXd z = Eigen::VectorXd::Zero(g.mgpi.consStif[L].rows());
        g.mgpi.MULT_VCYC(L, g.consForc, z, ds);
        save_vec("vcycle_z", z);
    }
    std::vector<double> info = {t_setup};
    if (do_cg) {
        Eigen::VectorXd x1, x0;
        double t1 = now_s();
        long it1 = capture_iters([&] { g.mgpi.CG_SOLV(1, g.consForc, x1); });
        double t_cg1 = now_s() - t1;
        save_vec("x_mg", x1);
        Eigen::VectorXd out;
        g.OUTP_SUB1(x1, out);
        save_vec("u_nodal", out);
        double t2 = now_s();
        long it0 = capture_iters([&] { g.mgpi.CG_SOLV(0, g.consForc, x0); });
        double t_cg0 = now_s() - t2;
        save_vec("x_diag", x0);
        Eigen::VectorXd r = g.consForc - g.mgpi.consStif[L] * x1;
        info.insert(info.end(), {(double)it1, t_cg1, (double)it0, t_cg0,
                                 r.norm() / g.consForc.norm()});
    }
    save_dvec("info", info);  // [t_setup, it_mg, t_mg, it_diag, t_diag, true_relres_mg]
    std::printf("beam_nodd n=%ld levels=%ld info:", (long)g.mgpi.consStif[L].rows(), L + 1);
    for (double v : info) std::printf(" %.6g", v);
    std::printf("\n");
    return 0;
}

// The other drivers of the MGPIS class surface on the BEAM mesh: MULT_SOLV (MGPIS.h:130-160),
// BiCGSTAB_SOLV(0/1) (MGPIS.h:350-432), GMRES_SOLV(0/1) (MGPIS.h:228-348).  Saves each solution,
// the last "#Iteration" value each printed and the true relative residual.
int beam_solv(long d0, long d1, long d2, long gl) {
    BEAM beam(0);
    beam.diviNumb = {d0, d1, d2};
    beam.globLeve = gl;
    quiet([&] { beam.MESH_NODD(0); });
    MULTIGRID& g = beam.multGrid[0];
    quiet([&] { g.TRANSFER(); g.STIF_MATR(); g.CONSTRAINT(1); });
    const long L = g.mgpi.maxiLeve;
    const Eigen::VectorXd& b = g.consForc;
    std::vector<double> info;
    auto run = [&](const char* name, auto fn) {
        Eigen::VectorXd x;
        long last = capture_iters([&] { fn(x); }) - 1;  // the printed value
        save_vec(name, x);
        Eigen::VectorXd r = b - g.mgpi.consStif[L] * x;
        info.push_back((double)last);
        info.push_back(r.norm() / b.norm());
    };
    run("x_mult", [&](Eigen::VectorXd& x) { g.mgpi.MULT_SOLV(b, x); });
    run("x_bicg1", [&](Eigen::VectorXd& x) { g.mgpi.BiCGSTAB_SOLV(1, b, x); });
    run("x_bicg0", [&](Eigen::VectorXd& x) { g.mgpi.BiCGSTAB_SOLV(0, b, x); });
    run("x_gmres1", [&](Eigen::VectorXd& x) { g.mgpi.GMRES_SOLV(1, b, x); });
    run("x_gmres0", [&](Eigen::VectorXd& x) { g.mgpi.GMRES_SOLV(0, b, x); });
    save_vec("consForc", b);
    save_dvec("solv_info", info);  // [printed iteration, true relres] per solver, order as above
    std::printf("beam_solv n=%ld info:", (long)b.size());
    for (double v : info) std::printf(" %.6g", v);
    std::printf("\n");
    return 0;
}

// Dump everything of an MCONTACT after CONTACT_ANALYSIS (MCONTACT.h:9-95 public members).
void dump_mcontact(MCONTACT& mc, const std::string& moni_path) {
    const long nsub = (long)mc.multGrid.size(), nint = (long)mc.searCont.size();
    save_ivec("n_sub_int", {nsub, nint, mc.iterNumbReco});
    for (long tv = 0; tv < nsub; ++tv) {
        std::string pre = "sd" + std::to_string(tv) + "_";
        dump_grid(pre, mc.multGrid[tv], false);
        save_csr(pre + "KL", mc.multGrid[tv].mgpi.consStif[mc.multGrid[tv].mgpi.maxiLeve]);
        save_vec(pre + "resuDisp", mc.resuDisp[tv]);
    }
    for (long ts = 0; ts < nint; ++ts) {
        std::string pre = "if" + std::to_string(ts) + "_";
        const auto& ips = mc.searCont[ts].intePoin;
        const size_t n = ips.size();
        std::vector<int64_t> node;
        std::vector<double> shap, basis, gap, w, cont;
        for (const auto& ip : ips) {
            for (int s = 0; s < 2; ++s) for (int k = 0; k < 4; ++k) node.push_back(ip.node[s][k]);
            for (int s = 0; s < 2; ++s) for (int k = 0; k < 4; ++k) shap.push_back(ip.shapFunc[s][k]);
            for (int b = 0; b < 3; ++b) for (int k = 0; k < 3; ++k) basis.push_back(ip.basiVect[b](k));
            for (int s = 0; s < 2; ++s) for (int k = 0; k < 3; ++k) cont.push_back(ip.contPoin[s](k));
            gap.push_back(ip.initNgap);
            w.push_back(ip.quadWeig);
        }
        save_npy(P(pre + "ip_node"), node.data(), {n, 2, 4});
        save_npy(P(pre + "ip_shap"), shap.data(), {n, 2, 4});
        save_npy(P(pre + "ip_basis"), basis.data(), {n, 3, 3});
        save_npy(P(pre + "ip_cont"), cont.data(), {n, 2, 3});
        save_dvec(pre + "ip_gap", gap);
        save_dvec(pre + "ip_w", w);
        save_dvec(pre + "param", {mc.fricCoef[ts], mc.penaFact_n[ts], mc.penaFact_f[ts]});
        save_ivec(pre + "body", {mc.contBody[ts][0], mc.contBody[ts][1]});
        for (int s = 0; s < 2; ++s) {
            std::string ps = pre + "s" + std::to_string(s) + "_";
            save_csr(ps + "systTran", mc.systTran[ts][s]);
            save_csr(ps + "systTran_pena", mc.systTran_pena[ts][s]);
            save_csr(ps + "inteMass", mc.inteMass[ts][s]);
            save_csr(ps + "inteMass_pena", mc.inteMass_pena[ts][s]);
            save_csr(ps + "inpoLagr", mc.inpoLagr[ts][s]);
            save_csr(ps + "inpoDisp", mc.inpoDisp[ts][s]);
            save_csr(ps + "inteInpo", mc.inteInpo[ts][s]);
            save_csr(ps + "pemaInpo_r", mc.pemaInpo_r[ts][s]);
            save_csr(ps + "systMass", mc.systMass[ts][s]);
            save_vec(ps + "inteAuxi", mc.inteAuxi[ts][s]);
            save_vec(ps + "inteLagr", mc.inteLagr[ts][s]);
            std::vector<int64_t> nc(mc.nodeCont[ts][s].size());
            for (const auto& kv : mc.nodeCont[ts][s]) nc[kv.second] = kv.first;
            save_ivec(ps + "nodeCont", nc);
        }
        save_vec(pre + "inpoNgap", mc.inpoNgap[ts]);
        // final projected gamma as written by OUTPUT_PRTR (MCONTACT.h:97-123)
        std::ifstream f(DIRECTORY("resuCont_" + std::to_string(ts) + ".txt"));
        std::vector<double> cont_out;
        double v;
        while (f >> v) cont_out.push_back(v);
        save_dvec(pre + "resuCont", cont_out);
    }
    if ((mc.muscSett >> 1) % 2 == 1) {
        save_csr("globCoup_1", mc.globCoup_1);
        save_vec("globForc_1", mc.globForc_1);
        std::vector<int64_t> base(mc.baseReco.begin(), mc.baseReco.end());
        save_ivec("baseReco", base);
        std::vector<int64_t> dole(mc.doleMcsc.begin(), mc.doleMcsc.end());
        save_ivec("doleMcsc", dole);
        for (long tv = 0; tv < nsub; ++tv) {
            save_csr("sd" + std::to_string(tv) + "_globTran_D_1", mc.globTran_D_1[tv]);
            save_csr("sd" + std::to_string(tv) + "_accuProl", mc.accuProl[tv]);
        }
        for (long ts = 0; ts < nint; ++ts)
            for (int s = 0; s < 2; ++s)
                save_csr("if" + std::to_string(ts) + "_s" + std::to_string(s) + "_globTran_1", mc.globTran_1[ts][s]);
    }
    if ((mc.muscSett >> 0) % 2 == 1) {  // LATIN-type coarse space (MULTISCALE, MCONTACT.h:898-1536)
        save_csr("globCoup", mc.globCoup);
        std::vector<int64_t> base(mc.baseReco.begin(), mc.baseReco.end());
        save_ivec("baseReco", base);
        std::vector<int64_t> dole(mc.doleMcsc.begin(), mc.doleMcsc.end());
        save_ivec("doleMcsc", dole);
        for (long tv = 0; tv < nsub; ++tv) save_csr("sd" + std::to_string(tv) + "_accuProl", mc.accuProl[tv]);
        for (long ts = 0; ts < nint; ++ts)
            for (int s = 0; s < 2; ++s) {
                const std::string ps = "if" + std::to_string(ts) + "_s" + std::to_string(s) + "_";
                save_csr(ps + "globTran", mc.globTran[ts][s]);
                save_csr(ps + "globTran_pena", mc.globTran_pena[ts][s]);
                save_csr(ps + "globTran_D", mc.globTran_D[ts][s]);
            }
    }
    save_ivec("muscSett", {mc.muscSett});
    // resuMoni.txt (MCONTACT.h:2742-2836): one row per ADMM iteration
    std::ifstream f(moni_path);
    std::vector<double> rows;
    std::string line;
    size_t ncol = 0, nrow = 0;
    while (std::getline(f, line)) {
        std::stringstream ls(line);
        double v;
        size_t c = 0;
        while (ls >> v) { rows.push_back(v); ++c; }
        if (c) { ncol = c; ++nrow; }
    }
    save_npy(P("resuMoni"), rows.data(), {nrow, ncol});
}

int beam_dd(long d0, long d1, long d2, long gl, long D0, long D1, long D2, long musc) {
    BEAM beam(1);
    beam.diviNumb = {d0, d1, d2};
    beam.globLeve = gl;
    beam.domaNumb = {D0, D1, D2};
    beam.muscSett = musc;
    beam.doleMcsc.clear();
    if (musc) beam.doleMcsc.assign(D0 * D1 * D2, 1);
    double t0 = now_s();
    std::string log;
    capture_iters([&] { beam.SOLVE(1, 1, 0); }, &log);
    double t = now_s() - t0;
    dump_mcontact(beam, DIRECTORY("resuMoni.txt"));
    std::printf("beam_dd subdomains=%zu interfaces=%zu iters=%ld wall=%.3fs\n",
                beam.multGrid.size(), beam.searCont.size(), beam.iterNumbReco, t);
    return 0;
}

// Box mesh in the reference's own data structures: nodes by TRY_ADD_NODE in (i,j,k) loop
// order, hexes with BLOCK.h's corner convention, uniform octree refinement (refiPatt 0) by
// MULTIGRID::REFINE, exactly like the examples' MESH routines do.
void box_mesh(MULTIGRID& g, double x0, double x1, double y0, double y1, double z0, double z1,
              long nx, long ny, long nz, long gl) {
    std::vector<long> id((nx + 1) * (ny + 1) * (nz + 1));
    auto I = [&](long i, long j, long k) { return (i * (ny + 1) + j) * (nz + 1) + k; };
    for (long i = 0; i <= nx; ++i)
        for (long j = 0; j <= ny; ++j)
            for (long k = 0; k <= nz; ++k)
                id[I(i, j, k)] = g.TRY_ADD_NODE(COOR(x0 + (x1 - x0) / nx * i, y0 + (y1 - y0) / ny * j,
                                                    z0 + (z1 - z0) / nz * k));
    for (long i = 0; i < nx; ++i)
        for (long j = 0; j < ny; ++j)
            for (long k = 0; k < nz; ++k) {
                TREE_ELEM e;
                e.parent = -1;
                e.cornNode = {id[I(i, j, k)], id[I(i + 1, j, k)], id[I(i + 1, j + 1, k)], id[I(i, j + 1, k)],
                              id[I(i, j, k + 1)], id[I(i + 1, j, k + 1)], id[I(i + 1, j + 1, k + 1)],
                              id[I(i, j + 1, k + 1)]};
                e.level = 0;
                e.refiPatt = 7;
                g.ADD_ELEMENT(e);
            }
    std::set<long> spl;
    std::map<long, std::set<long>> flag;
    std::map<std::vector<long>, COOR> plan;
    for (long r = 0; r < gl; ++r) {
        spl.clear();
        for (long t = 0; t < (long)g.elemVect.size(); ++t)
            if (g.elemVect[t].children.empty()) { spl.insert(t); g.elemVect[t].refiPatt = 0; }
        g.REFINE(spl, flag, plan);
    }
    g.coupReps = -1;
}

// Consistent nodal load of a uniform traction t on every element face lying in plane z = zc.
void face_traction(MULTIGRID& g, double zc, const Eigen::Vector3d& t) {
    for (const auto& el : g.elemVect) {
        if (!el.children.empty()) continue;
        for (const auto& f : hexaFace) {
            bool on = true;
            std::vector<Eigen::Vector3d> c(4);
            for (int k = 0; k < 4; ++k) {
                const COOR& p = g.nodeCoor.at(el.cornNode[f[k]]);
                c[k] << p[0], p[1], p[2];
                if (std::abs(p[2] - zc) > 1e-12) on = false;
            }
            if (!on) continue;
            double area = 0.5 * ((c[2] - c[0]).cross(c[3] - c[1])).norm();
            for (int k = 0; k < 4; ++k)
                for (int d = 0; d < 3; ++d) g.LOAD_ACCU(3 * el.cornNode[f[k]] + d, t(d) * area / 4.0);
        }
    }
}

// Two stacked blocks up to and including CONTACT_SEARCH (ESTABLISH / CONTACT_ANALYSIS left to
// the caller).  mc must stay in place: the search keeps pointers to its grids.
void twoblock_build(MCONTACT& mc, double fric, long gl) {
    mc.multGrid.resize(2);
    const double L = 0.02, H = 0.01, p = 1.0e7;
    box_mesh(mc.multGrid[0], 0, L, 0, L, 0, H, 2, 2, 1, gl);       // lower block (master)
    box_mesh(mc.multGrid[1], 0, L, 0, L, H, 2 * H, 2, 2, 1, gl);   // upper block (slave)
    for (int b = 0; b < 2; ++b) {
        MULTIGRID& g = mc.multGrid[b];
        for (const auto& it : g.nodeCoor) {  // rollers: x=0 -> ux, y=0 -> uy; bottom of A -> uz
            const COOR& c = it.second;
            if (c[0] <= 1e-12 && (b == 0 || fric == 0.0)) g.consDofv.emplace(3 * it.first + 0, 0.0);
            if (c[1] <= 1e-12) g.consDofv.emplace(3 * it.first + 1, 0.0);
            if (b == 0 && c[2] <= 1e-12) g.consDofv.emplace(3 * it.first + 2, 0.0);
        }
    }
    Eigen::Vector3d trac(fric > 0 ? 0.5 * fric * p : 0.0, 0.0, -p);
    face_traction(mc.multGrid[1], 2 * H, trac);
    // contact surface z = H (CURVEDS point set on the fine lattice)
    const long nf = 2L * (1L << gl);  // fine faces per side of the contact plane
    CURVEDS surf;
    surf.indiPoin.resize(nf + 1);
    for (long i = 0; i <= nf; ++i) {
        surf.indiPoin[i].resize(nf + 1);
        for (long j = 0; j <= nf; ++j) surf.INSERT(i, j, COOR(L / nf * i, L / nf * j, H));
    }
    mc.muscSett = 0;
    mc.doleMcsc.clear();
    std::string log;
    double charLeng = 0;
    capture_iters([&] { charLeng = mc.GET_CHAR_LENG(); }, &log);
    mc.searCont.resize(1);
    mc.contBody = {{0, 1}};
    mc.fricCoef = {fric};
    mc.penaFact_n = {210.0e9 * 25.0 / charLeng};
    mc.penaFact_f = {210.0e9 * 25.0 / charLeng};
    CSEARCH& cs = mc.searCont[0];
    cs.mastGrid = &mc.multGrid[0];
    cs.slavGrid = &mc.multGrid[1];
    EFACE_SURFACE e0(cs.mastGrid, &surf);
    while (e0.INCREMENT() == 1) cs.mastSegm.emplace_back(e0.currNode);
    EFACE_SURFACE e1(cs.slavGrid, &surf);
    while (e1.INCREMENT() == 1) cs.slavSegm.emplace_back(e1.currNode);
    auto centroids = [&](const MULTIGRID& g, const VECTOR2L& segs) {
        VECTOR2D c(2);
        for (const auto& s : segs) {
            double a = 0, b = 0;
            for (int k = 0; k < 4; ++k) { a += g.nodeCoor.at(s[k])[0]; b += g.nodeCoor.at(s[k])[1]; }
            c[0].push_back(a / 4.0);
            c[1].push_back(b / 4.0);
        }
        return c;
    };
    capture_iters([&] {
        cs.BUCKET_SORT(centroids(mc.multGrid[0], cs.mastSegm), {nf, nf});
        cs.CONTACT_SEARCH(centroids(mc.multGrid[1], cs.slavSegm));
    }, &log);
}

int twoblock(double fric, long gl, long musc) {
    MCONTACT mc;
    twoblock_build(mc, fric, gl);
    mc.muscSett = musc;
    if (musc) mc.doleMcsc.assign(2, 1);
    std::string log;
    double t0 = now_s();
    capture_iters([&] {
        mc.ESTABLISH();
        mc.CONTACT_ANALYSIS();
    }, &log);
    double t = now_s() - t0;
    dump_mcontact(mc, DIRECTORY("resuMoni.txt"));
    std::printf("twoblock fric=%g ips=%zu iters=%ld wall=%.3fs\n", fric, mc.searCont[0].intePoin.size(),
                mc.iterNumbReco, t);
    return 0;
}

int time_cg(long d0, long d1, long d2, long gl, long reps) {
    BEAM beam(0);
    beam.diviNumb = {d0, d1, d2};
    beam.globLeve = gl;
    std::string log;
    MULTIGRID* gp = nullptr;
    double t0 = now_s();
    capture_iters([&] {
        beam.MESH_NODD(0);
        gp = &beam.multGrid[0];
        gp->TRANSFER(); gp->STIF_MATR(); gp->CONSTRAINT(1);
    }, &log);
    double t_setup = now_s() - t0;
    MULTIGRID& g = *gp;
    const long n = g.mgpi.consStif[g.mgpi.maxiLeve].rows();
    for (long r = 0; r < reps; ++r) {
        Eigen::VectorXd x;
        double t1 = now_s();
        long it = capture_iters([&] { g.mgpi.CG_SOLV(1, g.consForc, x); });
        double t = now_s() - t1;
        std::printf("{\"n\": %ld, \"levels\": %ld, \"iters\": %ld, \"cg_s\": %.6f, \"setup_s\": %.3f, "
                    "\"dof_iter_per_s\": %.6g, \"threads\": %d}\n",
                    n, g.mgpi.maxiLeve + 1, it, t, t_setup, (double)n * it / t, omp_get_max_threads());
        std::fflush(stdout);
    }
    return 0;
}

template <typename T>
std::vector<T> read_raw(const std::string& path, size_t n) {
    std::vector<T> v(n);
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f || std::fread(v.data(), sizeof(T), n, f) != n) throw std::runtime_error("cannot read " + path);
    std::fclose(f);
    return v;
}

Eigen::SparseMatrix<double, Eigen::RowMajor> read_csr(const std::string& pre, long rows, long cols, long nnz) {
    const auto p64 = read_raw<int64_t>(pre + ".ptr", rows + 1);
    auto col = read_raw<int32_t>(pre + ".col", nnz);
    auto val = read_raw<double>(pre + ".val", nnz);
    if (p64[0] != 0 || p64[rows] != nnz) throw std::runtime_error(pre + ": row pointer");
    std::vector<int> ptr(p64.begin(), p64.end());
    Eigen::Map<const Eigen::SparseMatrix<double, Eigen::RowMajor>> m(rows, cols, nnz, ptr.data(), col.data(), val.data());
    return Eigen::SparseMatrix<double, Eigen::RowMajor>(m);
}

int time_cg_ops(const std::string& dir, long reps) {
    std::ifstream meta(dir + "/meta.txt");
    long nlev = 0;
    if (!(meta >> nlev) || nlev < 1) throw std::runtime_error("meta.txt");
    MGPIS mg;
    mg.maxiLeve = nlev - 1;
    for (long l = 0; l < nlev; ++l) {
        long r, c, z;
        meta >> r >> c >> z;
        mg.consStif.push_back(read_csr(dir + "/K" + std::to_string(l), r, c, z));
    }
    for (long l = 0; l + 1 < nlev; ++l) {
        long r, c, z;
        meta >> r >> c >> z;
        mg.realProl.push_back(read_csr(dir + "/P" + std::to_string(l), r, c, z));
    }
    const long n = mg.consStif.back().rows();
    const auto bv = read_raw<double>(dir + "/b.f64", n);
    const Eigen::VectorXd b = Eigen::Map<const Eigen::VectorXd>(bv.data(), n);
    quiet([&] { mg.ESTABLISH(); });  // consLowe / consDiag / consUppe (MGPIS.h:36-49), setup
    for (long r = 0; r < reps; ++r) {
        Eigen::VectorXd x;
        const double t1 = now_s();
        const long it = capture_iters([&] { mg.CG_SOLV(1, b, x); });
        const double t = now_s() - t1;
        const double bn = b.norm(), rel = bn > 0 ? (b - mg.consStif.back() * x).norm() / bn : 0.0;
        std::printf("{\"n\": %ld, \"levels\": %ld, \"iters\": %ld, \"cg_s\": %.6f, \"true_relres\": %.3e, \"threads\": %d}\n",
                    n, nlev, it, t, rel, omp_get_max_threads());
        std::fflush(stdout);
    }
    return 0;
}

}  // namespace harness

#ifndef HARNESS_NO_MAIN
int main(int argc, char** argv) {
    using namespace harness;
    if (argc < 2) { std::fprintf(stderr, "usage: see header\n"); return 2; }
    std::string mode = argv[1];
    auto L = [&](int i) { return std::stol(argv[i]); };
    if (mode == "beam_nodd" && argc >= 8) {
        g_out = argv[6];
        return beam_nodd(L(2), L(3), L(4), L(5), L(7) != 0, argc >= 9 ? L(8) != 0 : true);
    }
    if (mode == "beam_dd" && argc >= 10) {
        g_out = argv[9];
        return beam_dd(L(2), L(3), L(4), L(5), L(6), L(7), L(8), argc >= 11 ? L(10) : 0);
    }
    if (mode == "twoblock" && argc >= 5) {
        g_out = argv[4];
        return twoblock(std::stod(argv[2]), L(3), argc >= 6 ? L(5) : 0);
    }
    if (mode == "time_cg" && argc >= 7) return time_cg(L(2), L(3), L(4), L(5), L(6));
    if (mode == "time_cg_ops" && argc >= 4) return time_cg_ops(argv[2], L(3));
    if (mode == "beam_solv" && argc >= 7) {
        g_out = argv[6];
        return beam_solv(L(2), L(3), L(4), L(5));
    }
    std::fprintf(stderr, "bad arguments\n");
    return 2;
}
#endif  // HARNESS_NO_MAIN
