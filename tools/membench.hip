// Memory-path microbenchmarks for the roofline views of bench.py:
//
//  mb_stream_x4     streaming dwordx4 read of a buffer far larger than the 256 MiB Infinity Cache:
//                   the guide's calibrated case (FETCH_SIZE = 1/2 of the bytes on gfx950)
//  mb_gather80_pad  every 80-B record of a table far larger than the MALL read once, in random
//                   order, each record alone in its 128-B line (5 x dwordx4 per lane, as the
//                   trajectory kernel's level-pair record reads): DRAM bytes known = 128 per record
//  mb_gather80      the same records packed at 80-B stride (the engine's layout): 80..160 B per
//                   record depending on whether a line's other record is still cached
//  mb_l1_x4         every lane re-reads its block's private 4 KiB with dwordx4 loads (all L1 hits):
//                   the vector-L1 / texture-data (TD) return rate per CU, the roof of a kernel
//                   whose gathers hit L1
//  mb_l1_bcast      the same, every lane of a wave reading the same 16 B (broadcast)
//
// Each kernel's bytes (to the lanes, and compulsory from DRAM) and its hipEvent time are printed as
// one JSON object; rocprofv3 --pmc passes over the same binary give FETCH_SIZE, TD_TD_BUSY_sum,
// TD_TD_SP_TRAFFIC_sum and GRBM_GUI_ACTIVE per kernel (tools/membench.sh).
//
//   hipcc --offload-arch=gfx950 -O3 -o build/membench tools/membench.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

__global__ void __launch_bounds__(256) mb_stream_x4(const double2* __restrict__ a, int64_t n, double* out) {
    double s = 0.0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const double2 v = a[i];
        s += v.x + v.y;
    }
    out[(int64_t)blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// record r at rec + r * stride_d doubles (10 doubles = 80 B read as 5 x 16 B)
__global__ void __launch_bounds__(256) mb_gather80(const double* __restrict__ rec, int64_t stride_d,
                                                   const uint32_t* __restrict__ perm, int64_t n, double* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double2* r = reinterpret_cast<const double2*>(rec + (int64_t)perm[i] * stride_d);
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        const double2 v = r[q];
        s += v.x + v.y;
    }
    out[i] = s;
}

__global__ void __launch_bounds__(256) mb_gather80_pad(const double* __restrict__ rec, int64_t stride_d,
                                                       const uint32_t* __restrict__ perm, int64_t n, double* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double2* r = reinterpret_cast<const double2*>(rec + (int64_t)perm[i] * stride_d);
    double s = 0.0;
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        const double2 v = r[q];
        s += v.x + v.y;
    }
    out[i] = s;
}

// each block: its own 4 KiB (256 x 16 B), read `iters` times; lane j of the block reads piece
// (j + k) % 256 at iteration k (16 B per lane per load, whole 1-KiB wave-instructions)
__global__ void __launch_bounds__(256) mb_l1_x4(const double2* __restrict__ a, int iters, double* out) {
    const double2* base = a + (int64_t)blockIdx.x * 256;
    double s = 0.0;
    for (int k = 0; k < iters; k += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const double2 v = base[(threadIdx.x + 64 * u + k) & 255];
            s += v.x + v.y;
        }
    }
    out[(int64_t)blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) mb_l1_bcast(const double2* __restrict__ a, int iters, double* out) {
    const double2* base = a + (int64_t)blockIdx.x * 256;
    double s = 0.0;
    const int w = threadIdx.x >> 6;
    for (int k = 0; k < iters; k += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const double2 v = base[(w * 64 + u + k) & 255];  // one address per wave-instruction
            s += v.x + v.y;
        }
    }
    out[(int64_t)blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// the same L1-resident re-reads with only some lanes of each wave active: mode 0 = 16 lanes spread
// (every 4th), 1 = 16 contiguous lanes, 2 = 48 lanes, 3 = 1 lane -- does the TD return cost scale
// with the active lanes of a wave-instruction?
__global__ void __launch_bounds__(256) mb_l1_partial(const double2* __restrict__ a, int iters, int mode, double* out) {
    const double2* base = a + (int64_t)blockIdx.x * 256;
    const int lane = threadIdx.x & 63;
    const bool on = mode == 0 ? (lane & 3) == 0 : mode == 1 ? lane < 16 : mode == 2 ? lane < 48 : lane == 0;
    double s = 0.0;
    if (on) {
        for (int k = 0; k < iters; k += 4) {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const double2 v = base[(threadIdx.x + 64 * u + k) & 255];
                s += v.x + v.y;
            }
        }
    }
    out[(int64_t)blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// does the TD cost of a wave-instruction grow with the distinct cache lines its lanes touch?  Each block
// re-reads its own 8 KiB (512 x 16 B, L1-resident at 2 blocks per CU); lane j reads piece
// (j * stride + k) & 511: stride 1 = 64 consecutive pieces (8 lines of 128 B), 2 = 16 lines, 4 = 32, 8 = 64
// (one line per lane) -- the trajectory kernel's record gathers are the last case
__global__ void __launch_bounds__(256) mb_l1_scatter(const double2* __restrict__ a, int iters, int stride, double* out) {
    const double2* base = a + (int64_t)blockIdx.x * 512;
    const int j = threadIdx.x & 63, w = threadIdx.x >> 6;
    double s = 0.0;
    for (int k = 0; k < iters; k += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const double2 v = base[(j * stride + 64 * (w + u) + k) & 511];
            s += v.x + v.y;
        }
    }
    out[(int64_t)blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static float time_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 3;
    int dev = 0, ncu = 0;
    CK(hipSetDevice(dev));
    CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    double* out = nullptr;
    const int64_t out_n = 1 << 26;
    CK(hipMalloc(&out, out_n * sizeof(double)));

    // 1. streaming read, 4 GiB
    const int64_t sn = (4ll << 30) / 16;
    double2* sbuf = nullptr;
    CK(hipMalloc(&sbuf, sn * 16));
    CK(hipMemset(sbuf, 0, sn * 16));
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0));
        mb_stream_x4<<<ncu * 8, 256>>>(sbuf, sn, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        printf("{\"kernel\": \"mb_stream_x4\", \"rep\": %d, \"ms\": %.4f, \"lane_bytes\": %lld, \"dram_bytes\": %lld}\n",
               r, time_ms(e0, e1), (long long)(sn * 16), (long long)(sn * 16));
    }
    CK(hipFree(sbuf));

    // 2./3. 80-B records, 2^25 of them (2.7 GB packed, 4.3 GB padded), random order, each once
    const int64_t nrec = 1ll << 25;
    std::vector<uint32_t> perm(nrec);
    for (int64_t i = 0; i < nrec; ++i) perm[i] = (uint32_t)i;
    uint64_t x = 88172645463325252ull;
    for (int64_t i = nrec - 1; i > 0; --i) {  // Fisher-Yates, xorshift64
        x ^= x << 13; x ^= x >> 7; x ^= x << 17;
        const int64_t j = (int64_t)(x % (uint64_t)(i + 1));
        const uint32_t t = perm[i]; perm[i] = perm[j]; perm[j] = t;
    }
    uint32_t* dperm = nullptr;
    CK(hipMalloc(&dperm, nrec * 4));
    CK(hipMemcpy(dperm, perm.data(), nrec * 4, hipMemcpyHostToDevice));
    double* out2 = nullptr;
    CK(hipMalloc(&out2, nrec * sizeof(double)));
    for (int pad = 1; pad >= 0; --pad) {
        const int64_t stride_d = pad ? 16 : 10;  // 128-B or 80-B record stride
        double* rec = nullptr;
        CK(hipMalloc(&rec, nrec * stride_d * 8));
        CK(hipMemset(rec, 0, nrec * stride_d * 8));
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            if (pad) mb_gather80_pad<<<(unsigned)((nrec + 255) / 256), 256>>>(rec, stride_d, dperm, nrec, out2);
            else mb_gather80<<<(unsigned)((nrec + 255) / 256), 256>>>(rec, stride_d, dperm, nrec, out2);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            // compulsory DRAM bytes: padded = one 128-B line per record; packed = the table once
            // (a line's second record may have to fetch it again: the FETCH_SIZE pass tells)
            printf("{\"kernel\": \"%s\", \"rep\": %d, \"ms\": %.4f, \"lane_bytes\": %lld, \"dram_bytes\": %lld, "
                   "\"records\": %lld}\n",
                   pad ? "mb_gather80_pad" : "mb_gather80", r, time_ms(e0, e1), (long long)(nrec * 80),
                   (long long)(pad ? nrec * 128 : nrec * 80), (long long)nrec);
        }
        CK(hipFree(rec));
    }
    CK(hipFree(dperm));
    CK(hipFree(out2));

    // 4./5. L1-resident re-reads: 8 blocks per CU, 4 KiB each
    const int nblk = ncu * 8;
    const int iters = 4096;
    double2* l1 = nullptr;
    CK(hipMalloc(&l1, (int64_t)nblk * 256 * 16));
    CK(hipMemset(l1, 0, (int64_t)nblk * 256 * 16));
    for (int r = 0; r < reps; ++r) {
        CK(hipEventRecord(e0));
        mb_l1_x4<<<nblk, 256>>>(l1, iters, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        printf("{\"kernel\": \"mb_l1_x4\", \"rep\": %d, \"ms\": %.4f, \"lane_bytes\": %lld, \"cus\": %d}\n", r,
               time_ms(e0, e1), (long long)nblk * 256 * iters * 16ll, ncu);
        CK(hipEventRecord(e0));
        mb_l1_bcast<<<nblk, 256>>>(l1, iters, out);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        printf("{\"kernel\": \"mb_l1_bcast\", \"rep\": %d, \"ms\": %.4f, \"lane_bytes\": %lld, \"cus\": %d}\n", r,
               time_ms(e0, e1), (long long)nblk * 256 * iters * 16ll, ncu);
    }
    for (int mode = 0; mode < 4; ++mode) {
        const int active = mode == 0 ? 16 : mode == 1 ? 16 : mode == 2 ? 48 : 1;
        for (int r = 0; r < reps; ++r) {
            CK(hipEventRecord(e0));
            mb_l1_partial<<<nblk, 256>>>(l1, iters, mode, out);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            printf("{\"kernel\": \"mb_l1_partial\", \"mode\": %d, \"active_lanes\": %d, \"rep\": %d, \"ms\": %.4f, "
                   "\"lane_bytes\": %lld, \"cus\": %d}\n", mode, active, r, time_ms(e0, e1),
                   (long long)nblk * 4 * active * iters * 16ll, ncu);
        }
    }
    CK(hipFree(l1));
    // 6. scattered L1-resident re-reads (mb_l1_scatter): 2 blocks per CU, 8 KiB each
    {
        const int nb2 = ncu * 2;
        double2* sc = nullptr;
        CK(hipMalloc(&sc, (int64_t)nb2 * 512 * 16));
        CK(hipMemset(sc, 0, (int64_t)nb2 * 512 * 16));
        for (int stride = 1; stride <= 8; stride *= 2) {
            for (int r = 0; r < reps; ++r) {
                CK(hipEventRecord(e0));
                mb_l1_scatter<<<nb2, 256>>>(sc, iters, stride, out);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                printf("{\"kernel\": \"mb_l1_scatter\", \"stride\": %d, \"lines_per_instr\": %d, \"rep\": %d, "
                       "\"ms\": %.4f, \"wave_instrs\": %lld, \"lane_bytes\": %lld, \"cus\": %d}\n", stride,
                       8 * stride, r, time_ms(e0, e1), (long long)nb2 * 4 * iters, (long long)nb2 * 256 * iters * 16ll,
                       ncu);
            }
        }
        CK(hipFree(sc));
    }
    CK(hipFree(out));
    return 0;
}
