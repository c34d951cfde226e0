// Prototype A/B (not product code): the fine PCG SpMV of the bench's lattice (8 members of
// 97 x 65 x 65 nodes, 27-point 3x3-block rows, lexicographic order) with
//   full : every block of a row streamed (the production SELL-BSR3 k_sell<kPcg> layout)
//   sym  : only the row's upper blocks (column >= row) streamed; the lower ones are the
//          transposes of blocks other rows store, read from those rows' slots (4-B slot index +
//          2-B column offset per entry) -- 0.58x the HBM bytes if those re-reads hit the caches.
// Both compute q = K z + beta q, p = z + beta p and the chunk partials of p.q; the results are
// compared and each variant timed with HIP events.
// Build: hipcc -O3 --offload-arch=gfx950 -o symspmv_proto symspmv_proto.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e), __FILE__, __LINE__); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

typedef double dbl2_t __attribute__((ext_vector_type(2)));
constexpr int C = 64;

__host__ __device__ inline int64_t elem(int ij, int64_t lane) { return ij == 8 ? 512 + lane : 128 * (ij / 2) + 2 * lane + ij % 2; }

template <bool NT, bool TR>
__device__ __forceinline__ void bfma(const double* sb, int lane, const double* xj, double& s0, double& s1, double& s2) {
    auto ld = [](const auto* p) { if constexpr (NT) return __builtin_nontemporal_load(p); else return *p; };
    const dbl2_t* p = reinterpret_cast<const dbl2_t*>(sb) + lane;
    const dbl2_t a = ld(p), b = ld(p + 64), c = ld(p + 128), d = ld(p + 192);
    const double v8 = ld(sb + 512 + lane);
    const double x0 = xj[0], x1 = xj[1], x2 = xj[2];
    if (!TR) {
        s0 += a.x * x0 + a.y * x1 + b.x * x2;
        s1 += b.y * x0 + c.x * x1 + c.y * x2;
        s2 += d.x * x0 + d.y * x1 + v8 * x2;
    } else {
        s0 += a.x * x0 + b.y * x1 + d.x * x2;
        s1 += a.y * x0 + c.x * x1 + d.y * x2;
        s2 += b.x * x0 + c.y * x1 + v8 * x2;
    }
}

struct Args {
    const int32_t* ns;     // per chunk: streamed slots
    const int64_t* off;    // per chunk: first slot
    const int16_t* c16;    // per slot lane
    const double* val;     // per slot 576 doubles
    const int32_t* nl;     // sym: per chunk lower entries
    const int64_t* loff;   // sym: per chunk first lower entry
    const int16_t* lc16;   // sym: per lower entry lane: column offset
    const int32_t* lpos;   // sym: per lower entry lane: slot index of K_ji in row j's storage
    int64_t nch;
    const int32_t* perm;   // per wave slot: chunk (-1 none), or null = identity
    const double* z;
    double* q;
    double* p;
    double* partial;
    double beta;
};

template <bool SYM, bool NTU, bool NTL, int WPB = 4>
__global__ __launch_bounds__(64 * WPB) void k_spmv(Args a) {
    const int lane = threadIdx.x & 63;
    int64_t c = (int64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
    if (a.perm) {
        c = a.perm[c];
        if (c < 0) return;
    } else if (c >= a.nch) return;
    const int64_t row = c * C + lane;
    double s0 = 0, s1 = 0, s2 = 0;
    const int ns = a.ns[c];
    const int64_t base = a.off[c];
#pragma unroll 3
    for (int k = 0; k < ns; ++k) {
        const int64_t j = row + __builtin_nontemporal_load(a.c16 + (base + k) * C + lane);
        bfma<NTU, false>(a.val + (base + k) * 576, lane, a.z + 3 * j, s0, s1, s2);
    }
    if (SYM) {
        const int nl = a.nl[c];
        const int64_t lb = a.loff[c];
#pragma unroll 3
        for (int k = 0; k < nl; ++k) {
            const int64_t j = row + __builtin_nontemporal_load(a.lc16 + (lb + k) * C + lane);
            const int64_t pos = __builtin_nontemporal_load(a.lpos + (lb + k) * C + lane);
            bfma<NTL, true>(a.val + pos * 576, (int)(j & 63), a.z + 3 * j, s0, s1, s2);
        }
    }
    const int64_t o = 3 * row;
    const double be = a.beta;
    const double q0 = s0 + be * a.q[o], q1 = s1 + be * a.q[o + 1], q2 = s2 + be * a.q[o + 2];
    const double p0 = a.z[o] + be * a.p[o], p1 = a.z[o + 1] + be * a.p[o + 1], p2 = a.z[o + 2] + be * a.p[o + 2];
    a.q[o] = q0; a.q[o + 1] = q1; a.q[o + 2] = q2;
    a.p[o] = p0; a.p[o + 1] = p1; a.p[o + 2] = p2;
    double d = p0 * q0 + p1 * q1 + p2 * q2;
    for (int s = 32; s > 0; s >>= 1) d += __shfl_xor(d, s, 64);
    if (lane == 0) a.partial[c] = d;
}

// the full layout with a chosen slot unroll and a waves-per-EU floor (register budget)
template <int U, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void k_full_occ(Args a) {
    const int lane = threadIdx.x & 63;
    const int64_t c = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (c >= a.nch) return;
    const int64_t row = c * C + lane;
    double s0 = 0, s1 = 0, s2 = 0;
    const int ns = a.ns[c];
    const int64_t base = a.off[c];
#pragma unroll U
    for (int k = 0; k < ns; ++k) {
        const int64_t j = row + __builtin_nontemporal_load(a.c16 + (base + k) * C + lane);
        bfma<true, false>(a.val + (base + k) * 576, lane, a.z + 3 * j, s0, s1, s2);
    }
    const int64_t o = 3 * row;
    const double be = a.beta;
    const double q0 = s0 + be * a.q[o], q1 = s1 + be * a.q[o + 1], q2 = s2 + be * a.q[o + 2];
    const double p0 = a.z[o] + be * a.p[o], p1 = a.z[o + 1] + be * a.p[o + 1], p2 = a.z[o + 2] + be * a.p[o + 2];
    a.q[o] = q0; a.q[o + 1] = q1; a.q[o + 2] = q2;
    a.p[o] = p0; a.p[o + 1] = p1; a.p[o + 2] = p2;
    double d = p0 * q0 + p1 * q1 + p2 * q2;
    for (int s = 32; s > 0; s >>= 1) d += __shfl_xor(d, s, 64);
    if (lane == 0) a.partial[c] = d;
}

static uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ULL; x ^= x >> 33;
    return x;
}
static double rnd(uint64_t k) { return (double)(mix(k) >> 11) * (1.0 / 9007199254740992.0) - 0.5; }

// block (i, j) of the symmetric test matrix, row-major; K_ji = K_ij^T
static void block(int64_t i, int64_t j, double* v) {
    const int64_t lo = std::min(i, j), hi = std::max(i, j);
    double b[9];
    for (int e = 0; e < 9; ++e) b[e] = rnd((uint64_t)lo * 1000003ULL + (uint64_t)hi * 7919ULL + e);
    if (lo == hi) {
        for (int r = 0; r < 3; ++r)
            for (int cc = 0; cc < 3; ++cc) v[3 * r + cc] = 0.5 * (b[3 * r + cc] + b[3 * cc + r]) + (r == cc ? 30.0 : 0.0);
        return;
    }
    for (int r = 0; r < 3; ++r)
        for (int cc = 0; cc < 3; ++cc) v[3 * r + cc] = (i == lo) ? b[3 * r + cc] : b[3 * cc + r];
}

int main(int argc, char** argv) {
    const int nsub = argc > 1 ? atoi(argv[1]) : 8;
    const int reps = argc > 2 ? atoi(argv[2]) : 30;
    const int NX = 97, NY = 65, NZ = 65;
    const int64_t nloc = (int64_t)NX * NY * NZ, npad = (nloc + 63) / 64 * 64;
    const int64_t nn = npad * nsub, nch = nn / 64;
    // rows: sorted column lists
    std::vector<std::vector<int64_t>> cols(nn);
    for (int s = 0; s < nsub; ++s)
        for (int z = 0; z < NZ; ++z)
            for (int y = 0; y < NY; ++y)
                for (int x = 0; x < NX; ++x) {
                    const int64_t i = s * npad + ((int64_t)z * NY + y) * NX + x;
                    for (int dz = -1; dz <= 1; ++dz)
                        for (int dy = -1; dy <= 1; ++dy)
                            for (int dx = -1; dx <= 1; ++dx) {
                                const int X = x + dx, Y = y + dy, Z = z + dz;
                                if (X < 0 || Y < 0 || Z < 0 || X >= NX || Y >= NY || Z >= NZ) continue;
                                cols[i].push_back(s * npad + ((int64_t)Z * NY + Y) * NX + X);
                            }
                }
    for (int64_t i = 0; i < nn; ++i)
        if (cols[i].empty()) cols[i].push_back(i);  // pad rows: identity
    auto build = [&](bool sym, std::vector<int32_t>& ns, std::vector<int64_t>& off, std::vector<int16_t>& c16,
                     std::vector<double>& val, std::vector<int32_t>& nl, std::vector<int64_t>& loff,
                     std::vector<int16_t>& lc16, std::vector<int32_t>& lpos) {
        ns.assign(nch, 0);
        off.assign(nch + 1, 0);
        std::vector<int64_t> pos_of(sym ? 0 : 0);
        for (int64_t c = 0; c < nch; ++c) {
            int m = 0;
            for (int l = 0; l < 64; ++l) {
                const int64_t i = c * 64 + l;
                int k = 0;
                for (int64_t j : cols[i]) k += (!sym || j >= i);
                m = std::max(m, k);
            }
            ns[c] = m;
            off[c + 1] = off[c] + m;
        }
        const int64_t nsl = off[nch] + 1;  // + one zero slot
        c16.assign(nsl * 64, 0);
        val.assign(nsl * 576, 0.0);
        // slot index of block (i -> j) in i's storage (upper part)
        std::vector<std::vector<int32_t>> slot_of(sym ? nn : 0);
        for (int64_t c = 0; c < nch; ++c)
            for (int l = 0; l < 64; ++l) {
                const int64_t i = c * 64 + l;
                int k = 0;
                for (int64_t j : cols[i]) {
                    if (sym && j < i) continue;
                    const int64_t sl = off[c] + k;
                    c16[sl * 64 + l] = (int16_t)(j - i);
                    double v[9];
                    block(i, j, v);
                    for (int e = 0; e < 9; ++e) val[sl * 576 + elem(e, l)] = v[e];
                    if (sym) slot_of[i].push_back((int32_t)sl);
                    ++k;
                }
            }
        if (!sym) return;
        nl.assign(nch, 0);
        loff.assign(nch + 1, 0);
        for (int64_t c = 0; c < nch; ++c) {
            int m = 0;
            for (int l = 0; l < 64; ++l) {
                const int64_t i = c * 64 + l;
                int k = 0;
                for (int64_t j : cols[i]) k += (j < i);
                m = std::max(m, k);
            }
            nl[c] = m;
            loff[c + 1] = loff[c] + m;
        }
        lc16.assign(loff[nch] * 64, 0);
        lpos.assign(loff[nch] * 64, (int32_t)off[nch]);  // pad: the zero slot, column = row
        for (int64_t c = 0; c < nch; ++c)
            for (int l = 0; l < 64; ++l) {
                const int64_t i = c * 64 + l;
                int k = 0;
                for (int64_t j : cols[i]) {
                    if (j >= i) continue;
                    // K_ij = (K_ji)^T; K_ji is in j's upper storage
                    int kk = 0;
                    for (int64_t t : cols[j]) {
                        if (t < j) continue;
                        if (t == i) break;
                        ++kk;
                    }
                    const int64_t e = (loff[c] + k) * 64 + l;
                    lc16[e] = (int16_t)(j - i);
                    lpos[e] = slot_of[j][kk];
                    ++k;
                }
            }
    };
    std::vector<int32_t> nsF, nsS, nlS, dummy32, lposS;
    std::vector<int64_t> offF, offS, loffS, dummy64;
    std::vector<int16_t> c16F, c16S, lc16S, dummy16;
    std::vector<double> valF, valS;
    build(false, nsF, offF, c16F, valF, dummy32, dummy64, dummy16, dummy32);
    build(true, nsS, offS, c16S, valS, nlS, loffS, lc16S, lposS);
    printf("nsub %d nodes %ld chunks %ld: full slots %ld (%.2f GB values), sym upper slots %ld lower %ld (%.2f GB)\n", nsub,
           (long)nn, (long)nch, (long)offF[nch], offF[nch] * 576 * 8e-9, (long)offS[nch], (long)loffS[nch],
           offS[nch] * 576 * 8e-9);
    // vectors
    std::vector<double> z(3 * nn), q0(3 * nn), p0(3 * nn);
    for (int64_t i = 0; i < 3 * nn; ++i) {
        z[i] = rnd(i * 3 + 1);
        q0[i] = rnd(i * 3 + 2);
        p0[i] = rnd(i * 3 + 3);
    }
    auto up = [](auto& v) {
        using T = typename std::decay_t<decltype(v)>::value_type;
        T* d = nullptr;
        CK(hipMalloc(&d, std::max<size_t>(1, v.size()) * sizeof(T)));
        if (!v.empty()) CK(hipMemcpy(d, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
        return d;
    };
    Args F{}, S{};
    F.ns = up(nsF); F.off = up(offF); F.c16 = up(c16F); F.val = up(valF); F.nch = nch;
    S.ns = up(nsS); S.off = up(offS); S.c16 = up(c16S); S.val = up(valS); S.nch = nch;
    S.nl = up(nlS); S.loff = up(loffS); S.lc16 = up(lc16S); S.lpos = up(lposS);
    valF.clear(); valF.shrink_to_fit(); valS.clear(); valS.shrink_to_fit();
    double *dz = up(z), *dq = up(q0), *dp = up(p0), *dpart = nullptr;
    CK(hipMalloc(&dpart, nch * sizeof(double)));
    F.z = S.z = dz; F.q = S.q = dq; F.p = S.p = dp; F.partial = S.partial = dpart;
    F.beta = S.beta = 0.0;  // beta = 0: q = K z, p = z (idempotent across reps)
    const int grid = (int)((nch + 3) / 4);
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> qF(3 * nn), qS(3 * nn);
    auto run = [&](const char* name, auto kern, const Args& A, double bytes, std::vector<double>* out, int g = 0, int bs = 256) {
        if (!g) g = grid;
        hipLaunchKernelGGL(kern, dim3(g), dim3(bs), 0, 0, A);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(kern, dim3(g), dim3(bs), 0, 0, A);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ms /= reps;
        printf("%-28s %8.4f ms  %6.3f GB  %6.2f TB/s algorithmic\n", name, ms, bytes * 1e-9, bytes / ms * 1e-9);
        if (out) CK(hipMemcpy(out->data(), dq, 3 * nn * 8, hipMemcpyDeviceToHost));
    };
    const double vec = 120.0 * nn;  // z gathered once, q and p read and written
    const double bF = offF[nch] * 64 * 74.0 + vec;
    const double bS = offS[nch] * 64 * 74.0 + loffS[nch] * 64 * 6.0 + vec;
    // XCD-band schedules: chunk -> (member, y band of its first row); band group t -> XCD t % 8;
    // each XCD walks its groups band by band, planes in order (one chunk per workgroup, WG b on
    // XCD b % 8 takes the (b / 8)-th chunk of that XCD's sequence)
    auto band_perm = [&](int B) {
        std::vector<std::vector<std::pair<int64_t, int64_t>>> seq(8);
        const int nb = (NY + B - 1) / B;
        for (int64_t c = 0; c < nch; ++c) {
            const int64_t r0 = c * 64, s_ = r0 / npad, l0 = r0 % npad;
            const int64_t z = l0 / ((int64_t)NX * NY), y = (l0 / NX) % NY;
            const int64_t t = s_ * nb + std::min<int64_t>(y / B, nb - 1);
            seq[t % 8].push_back({(t / 8) * (int64_t)1 << 40 | (z * NY + y) << 8, c});
        }
        size_t mx = 0;
        for (auto& v : seq) {
            std::sort(v.begin(), v.end());
            mx = std::max(mx, v.size());
        }
        std::vector<int32_t> perm(8 * mx, -1);
        for (int x = 0; x < 8; ++x)
            for (size_t k = 0; k < seq[x].size(); ++k) perm[8 * k + x] = (int32_t)seq[x][k].second;
        return perm;
    };
    std::vector<int32_t> pB4 = band_perm(4), pB8 = band_perm(8), pB16 = band_perm(16), pB65 = band_perm(65);
    auto upperm = [&](std::vector<int32_t>& v) { int32_t* d = nullptr; CK(hipMalloc(&d, v.size() * 4)); CK(hipMemcpy(d, v.data(), v.size() * 4, hipMemcpyHostToDevice)); return d; };
    int32_t *dB4 = upperm(pB4), *dB8 = upperm(pB8), *dB16 = upperm(pB16), *dB65 = upperm(pB65);
    if (argc > 3) {  // occupancy / unroll sweep of the full layout only
        for (int rep = 0; rep < 2; ++rep) {
            run("full (NT values)", k_spmv<false, true, true>, F, bF, &qF);
            run("full U3 wpe1", k_full_occ<3, 1>, F, bF, nullptr);
            run("full U3 wpe6", k_full_occ<3, 6>, F, bF, nullptr);
            run("full U3 wpe8", k_full_occ<3, 8>, F, bF, nullptr);
            run("full U2 wpe8", k_full_occ<2, 8>, F, bF, nullptr);
            run("full U4 wpe1", k_full_occ<4, 1>, F, bF, nullptr);
            run("full U6 wpe1", k_full_occ<6, 1>, F, bF, nullptr);
            run("full U1 wpe8", k_full_occ<1, 8>, F, bF, nullptr);
        }
        return 0;
    }
    for (int rep = 0; rep < 2; ++rep) {
        run("full (NT values)", k_spmv<false, true, true>, F, bF, &qF);
        run("full 1-wave WGs", k_spmv<false, true, true, 1>, F, bF, nullptr, (int)nch, 64);
        run("sym 1-wave WGs upC lowNT", k_spmv<true, false, true, 1>, S, bS, nullptr, (int)nch, 64);
        for (auto pr : {std::make_pair("B4", dB4), std::make_pair("B8", dB8), std::make_pair("B16", dB16), std::make_pair("B65", dB65)}) {
            const size_t np = pr.second == dB4 ? pB4.size() : pr.second == dB8 ? pB8.size() : pr.second == dB16 ? pB16.size() : pB65.size();
            Args X = S;
            X.perm = pr.second;
            char nm[64];
            snprintf(nm, sizeof nm, "sym xcd %s upC lowNT", pr.first);
            run(nm, k_spmv<true, false, true, 1>, X, bS, nullptr, (int)np, 64);
            snprintf(nm, sizeof nm, "sym xcd %s upC lowC", pr.first);
            run(nm, k_spmv<true, false, false, 1>, X, bS, &qS, (int)np, 64);
            Args Y = F;
            Y.perm = pr.second;
            snprintf(nm, sizeof nm, "full xcd %s", pr.first);
            run(nm, k_spmv<false, true, true, 1>, Y, bF, nullptr, (int)np, 64);
        }
        run("full (cached values)", k_spmv<false, false, false>, F, bF, nullptr);
        run("sym  upper NT, lower NT", k_spmv<true, true, true>, S, bS, &qS);
        run("sym  upper cached, lower NT", k_spmv<true, false, true>, S, bS, nullptr);
        run("sym  upper cached, lower cached", k_spmv<true, false, false>, S, bS, nullptr);
        run("sym  upper NT, lower cached", k_spmv<true, true, false>, S, bS, nullptr);
    }
    double md = 0, mx = 0;
    for (int64_t i = 0; i < 3 * nn; ++i) {
        md = std::max(md, std::fabs(qF[i] - qS[i]));
        mx = std::max(mx, std::fabs(qF[i]));
    }
    printf("max |q_full - q_sym| = %.3e (max |q| %.3e)\n", md, mx);
    return md <= 1e-12 * mx ? 0 : 3;
}
