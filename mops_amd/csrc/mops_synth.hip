// Synthetic MPAS-Ocean snapshot generator for the configs 4/5 bench (not part of
// the engine's ABI: it stands in for reading history files).  The analytic flow
// of mops_amd/synth.py:make_snapshot -- solid body + travelling wave-3, depth
// decay, w on the interface grid -- evaluated one cell per lane: the level
// recurrence (cumulative thickness) runs serially per lane in the same order as
// numpy's cumsum.
//
// Output rows are cell-major (row c = L levels), so a lane writing its own row
// stores 8 B per instruction 8*L bytes away from its neighbours: with ~2k lanes
// per CU in flight, the partially written lines outgrow the L2 and are evicted
// half-filled (masked HBM writes, ~470 GB/s measured).  Each wave therefore
// computes its 64 cells kSynthCh levels at a time into LDS and writes the chunk
// back as whole 128-B lines (lanes 0-15: cell 0's 16 levels, ...).  The
// interface velocity needs the column total, which a first pass over the levels
// computes with the same additions in the same order as the second.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cmath>

constexpr int kSynthCh = 16;  // levels per chunk: one 128-B line of a cell's row

__global__ void __launch_bounds__(64) synth_snapshot_kernel(int64_t C, int L, const double* __restrict__ lat_c,
                                                            const double* __restrict__ lon_c,
                                                            const double* __restrict__ ref_dz, double H, double phase,
                                                            double u0, double u1, double w0, double* __restrict__ thick,
                                                            double* __restrict__ bot_out, double* __restrict__ uo,
                                                            double* __restrict__ vo, double* __restrict__ wo) {
    __shared__ double s_t[64][kSynthCh + 1], s_u[64][kSynthCh + 1], s_v[64][kSynthCh + 1], s_w[64][kSynthCh + 1];
    const int lane = threadIdx.x;
    const int64_t c0 = (int64_t)blockIdx.x * 64;
    const int64_t c = c0 + lane;
    const int nc = (int)(C - c0 < 64 ? C - c0 : 64);
    const int64_t cr = c < C ? c : C - 1;  // lanes past the end compute a copy of the last cell, never stored
    const double lat = lat_c[cr], lon = lon_c[cr];
    double bot = H - 0.5 * (H - 2000.0) * (1.0 + sin(2.0 * lat) * cos(3.0 * lon)) * 0.5;
    bot = fmin(fmax(bot, 1500.0), H);
    if (c < C) bot_out[c] = bot;
    const double ssh = 0.5 * cos(lat) * sin(2.0 * lon + phase);
    const double scale = (bot + ssh) / H;
    const double cl = cos(lat);
    const double cu = u0 * cl + u1 * cos(3.0 * lon - phase) * sin(2.0 * lat) * cl;
    const double cv = u1 * sin(3.0 * lon - phase) * cl * cl;
    const double a = w0 * sin(2.0 * lat), b = cos(lon - phase);
    double total = 0.0;
    for (int k = 0; k < L; ++k) total += ref_dz[k] * scale;
    const int64_t W = (int64_t)L + 1;
    if (c < C) wo[c * W] = a * sin(M_PI * 0.0 / total) * b;
    double csum = 0.0;
    for (int k0 = 0; k0 < L; k0 += kSynthCh) {
        const int n = L - k0 < kSynthCh ? L - k0 : kSynthCh;
        for (int kk = 0; kk < n; ++kk) {
            const double tk = ref_dz[k0 + kk] * scale;
            csum += tk;
            const double decay = exp(-(csum - 0.5 * tk) / 1500.0);
            s_t[lane][kk] = tk;
            s_u[lane][kk] = cu * decay;
            s_v[lane][kk] = cv * decay;
            s_w[lane][kk] = a * sin(M_PI * csum / total) * b;  // interface k0 + kk + 1
        }
        __syncthreads();
        for (int idx = lane; idx < nc * n; idx += 64) {
            const int r = idx / n, kk = idx - r * n;
            const int64_t o = (c0 + r) * (int64_t)L + k0 + kk;
            thick[o] = s_t[r][kk];
            uo[o] = s_u[r][kk];
            vo[o] = s_v[r][kk];
            wo[(c0 + r) * W + k0 + kk + 1] = s_w[r][kk];
        }
        __syncthreads();
    }
}

extern "C" int mops_synth_snapshot(int64_t C, int L, const double* lat, const double* lon, const double* ref_dz,
                                   double H, double phase, double u0, double u1, double w0, double* thick,
                                   double* bot, double* u, double* v, double* wv, void* stream) {
    if (C <= 0 || L <= 0) return -1;
    const unsigned g = (unsigned)((C + 63) / 64);
    synth_snapshot_kernel<<<g, 64, 0, (hipStream_t)stream>>>(C, L, lat, lon, ref_dz, H, phase, u0, u1, w0, thick, bot,
                                                             u, v, wv);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// the source's identity, stamped by __graft_entry__.build_synth (rebuilt when it differs)
#ifndef MOPS_SYNTH_BUILD_ID
#define MOPS_SYNTH_BUILD_ID "unstamped"
#endif
extern "C" __attribute__((used)) const char* mops_synth_build_id() { return MOPS_SYNTH_BUILD_ID; }
