// Synthetic MPAS-Ocean snapshot generator for the configs 4/5 bench (not part of
// the engine's ABI: it stands in for reading history files).  The analytic flow
// of mops_amd/synth.py:make_snapshot -- solid body + travelling wave-3, depth
// decay, w on the interface grid -- evaluated in one pass per cell: the
// level recurrences (cumulative thickness) run serially per thread in the same
// order as numpy's cumsum, and every output row is written by its own thread.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cmath>

__global__ void __launch_bounds__(64) synth_snapshot_kernel(int64_t C, int L, const double* __restrict__ lat_c,
                                                            const double* __restrict__ lon_c,
                                                            const double* __restrict__ ref_dz, double H, double phase,
                                                            double u0, double u1, double w0, double* __restrict__ thick,
                                                            double* __restrict__ bot_out, double* __restrict__ uo,
                                                            double* __restrict__ vo, double* __restrict__ wo) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const double lat = lat_c[c], lon = lon_c[c];
    double bot = H - 0.5 * (H - 2000.0) * (1.0 + sin(2.0 * lat) * cos(3.0 * lon)) * 0.5;
    bot = fmin(fmax(bot, 1500.0), H);
    bot_out[c] = bot;
    const double ssh = 0.5 * cos(lat) * sin(2.0 * lon + phase);
    const double scale = (bot + ssh) / H;
    const double cl = cos(lat);
    const double cu = u0 * cl + u1 * cos(3.0 * lon - phase) * sin(2.0 * lat) * cl;
    const double cv = u1 * sin(3.0 * lon - phase) * cl * cl;
    double* t = thick + c * L;
    double* u = uo + c * L;
    double* v = vo + c * L;
    double* w = wo + c * (int64_t)(L + 1);
    double csum = 0.0;
    w[0] = 0.0;  // interface depths first; turned into w below once the column total is known
    for (int k = 0; k < L; ++k) {
        const double tk = ref_dz[k] * scale;
        t[k] = tk;
        csum += tk;
        const double decay = exp(-(csum - 0.5 * tk) / 1500.0);
        u[k] = cu * decay;
        v[k] = cv * decay;
        w[k + 1] = csum;
    }
    const double a = w0 * sin(2.0 * lat), b = cos(lon - phase);
    for (int j = 0; j <= L; ++j) w[j] = a * sin(M_PI * w[j] / csum) * b;
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
