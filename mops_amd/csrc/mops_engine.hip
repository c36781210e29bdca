// mops_engine.hip -- MI355X (gfx950, CDNA4) particle-trajectory engine.
//
// Hand-written HIP for the reference's StreamLine / PathLine hot path
// (YosefQiu/MOPS src/CPU/TBB/Kernel/MPASOVisualizerKernels.cpp:653-1496) and
// its derived-field producers (src/CPU/TBB/MPASOSolutionTBB.cpp).  Written for
// CDNA4 from the reference's semantics, not translated from its CUDA/HIP
// backend:
//
//  * one lane per particle, wave64, all steps of a segment inside one launch;
//    the particle state (position, float depth, cell) lives in registers and
//    the per-cell stencil (vertex ids, vertex coordinates, neighbour ids and
//    the polygon-only Wachspress terms B_i) is cached in registers across
//    steps -- a particle keeps its cell for ~10^3 steps at dt = 120 s;
//  * the mesh is re-laid out in HBM as one 64-B "cell record" per cell
//    (nEdges, 0-based verticesOnCell, 0-based cellsOnCell) plus 32-B padded
//    xyz rows, so every stencil fetch is whole sectors;
//  * the zTop column is never materialised: a streaming pass applies the
//    reference's monotone fix-up in order and derives the layer bracket from
//    two monotone predicates, stopping at the first level below the particle
//    (exactly the reference's result -- see bracket_scan);
//  * FP64 throughout with -ffp-contract=off and the reference's operation
//    order, so results are bit-comparable with the CPU path.
//
// No MFMA: this is a latency/bandwidth-bound gather.

#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <limits>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "mops_io.h"
#include "mops_traj.h"

#define MOPS_ABI_VERSION 4
#ifndef MOPS_BUILD_ID
#define MOPS_BUILD_ID "unstamped"  // __graft_entry__.build_engine passes the sources' identity (mops_build_id)
#endif

namespace {

thread_local std::string g_last_error;

mops_status fail(mops_status st, const std::string& msg) {
    g_last_error = msg;
    return st;
}

#define HIP_TRY(expr)                                                                   \
    do {                                                                                \
        hipError_t _e = (expr);                                                         \
        if (_e != hipSuccess)                                                           \
            return fail(MOPS_ERR_HIP, std::string(#expr " failed: ") + hipGetErrorString(_e)); \
    } while (0)

constexpr int kMaxLevels = 100;  // reference MAX_VERTICAL_LEVEL_NUM
constexpr int kMaxVertex = 20;   // reference MAX_VERTEX_NUM
constexpr int kBlock = 256;
#ifndef MOPS_TRAJ_BLOCK
#define MOPS_TRAJ_BLOCK 64  // one wave per workgroup: a slow wave never holds a block's slots
#endif
constexpr int kTrajBlock = MOPS_TRAJ_BLOCK;
constexpr int kPairRec = 10;  // doubles per level-pair record (see mops_field::d_pr)
#ifndef MOPS_PAIR_TEST
#define MOPS_PAIR_TEST 0  // the walk's pair test (dev::walk; superseded by dev::nbr_stay)
#endif
#ifndef MOPS_PAIR_TEST_P
#define MOPS_PAIR_TEST_P 0  // ... in the pathline kernels
#endif
// Compact per-lane LDS (traj_kernel): edge normals for polygon slots 0-5 only (slot 6, used by
// heptagons alone, is computed in the evaluation: same operands, same bits) and the pair-test
// radius as a float rounded toward zero (a smaller ball: the test stays conservative) --
// 11.5 KB per 64-lane block instead of 13 KB.  Fuller LDS measured slower even at the same
// 12 blocks per CU.
#ifndef MOPS_LDS_COMPACT
#define MOPS_LDS_COMPACT 1
#endif
#ifndef MOPS_NRM_SLOTS
#define MOPS_NRM_SLOTS 5  // polygon slots whose normals live in LDS (MOPS_LDS_COMPACT; slots 5-6 computed per evaluation)
#endif
constexpr int kNrmSlots(int maxv) { return (MOPS_LDS_COMPACT && maxv > MOPS_NRM_SLOTS) ? MOPS_NRM_SLOTS : maxv; }
// Level-pair record layout (mops_field::d_pr) in 16-B pieces: piece q (0..4) of the record of layer k1 = k-1
// and vertex v.  MOPS_PR_PIECES = 1 (round 5): piece-major [L-1][5][V+1] -- piece q of consecutive vertices is
// contiguous, and vertices are numbered in Morton order at mesh creation (MOPS_VPERM), so the lanes of one
// gather instruction, which ask for piece q of the records of neighbouring cells' vertices, share 128-B lines:
// the vector L1 / TD spends a cycle per distinct line of an instruction (tools/membench.hip mb_l1_scatter:
// 8-16 lines 17 cycles, 32 lines 33, 64 lines 64).  The all-zero record is vertex V of every (layer, piece).
// 0: record-major, level-major [L-1][V][5] (rounds 2-4) + one all-zero record after the last.
#ifndef MOPS_PR_PIECES
#define MOPS_PR_PIECES 0  // measured slower: record-major stays
#endif
#ifndef MOPS_VPERM
#define MOPS_VPERM 1  // mesh vertices renumbered internally in the Morton order of their coordinates
#endif
// (all in 16-B piece units; uint32 throughout: mops_mesh_create checks pr_pieces < 2^32)
__host__ __device__ __forceinline__ uint32_t pr_base(uint32_t k1, uint32_t v, uint32_t V) {  // piece 0
    return MOPS_PR_PIECES ? k1 * 5u * (V + 1u) + v : (k1 * V + v) * 5u;
}
__host__ __device__ __forceinline__ uint32_t pr_qstride(uint32_t V) { return MOPS_PR_PIECES ? V + 1u : 1u; }
__host__ __device__ __forceinline__ uint32_t pr_zero(uint32_t V, uint32_t L) {  // the all-zero record's piece 0
    return MOPS_PR_PIECES ? V : (L - 1u) * V * 5u;
}
inline uint64_t pr_pieces(int64_t V, int L) {
    return MOPS_PR_PIECES ? (uint64_t)(L - 1) * 5u * (uint64_t)(V + 1) : ((uint64_t)(L - 1) * (uint64_t)V + 1u) * 5u;
}

inline int rec_ints_for(int maxv) { return ((1 + 2 * maxv) + 3) / 4 * 4; }

// Cooperative waves (pathline Euler, MAXV 7): the pathline kernel is bound by the texture-data
// unit that returns VMEM data to the lanes (TD 96-98% busy at configs 3/4), because every lane
// gathers its own 12 level-pair records and 7 polygon slots although a wave's lanes share one to
// three cells.  A wave whose live lanes form at most MOPS_COOP_G groups of equal (cell, hinted
// front layer, hinted back layer) loads each group's polygon and records ONCE -- one 16-B piece
// per lane, the pieces of all groups spread over the wave -- into an LDS tile, and its lanes
// read them from there (ds_read_b128).  Same doubles, same order: bit-identical results.
#ifndef MOPS_FUSED_RECORDS
#define MOPS_FUSED_RECORDS 1  // derivation: vertex values computed inside the record build (field_derive)
#endif
#ifndef MOPS_COOP_PE
#define MOPS_COOP_PE 1
#endif
#ifndef MOPS_COOP_PR
#define MOPS_COOP_PR 1  // ... and pathline RK4
#endif
#ifndef MOPS_GR_COOP
#define MOPS_GR_COOP 2  // level-pair records per LDS round trip in the tile instantiations (1: +1%, 3: +7%)
#endif
#ifndef MOPS_COOP_R
#define MOPS_COOP_R 13  // tile pieces per live lane at most (fewer live lanes: the lanes gather themselves)
#endif
#ifndef MOPS_COOP_G
// groups per wave with a tile (LDS: 1296 B (6 tile slots) + an 80-B header each).  Round 6: with 7 tile slots,
// 8 groups (12.8 KB per block) still allow the 12 blocks per CU the kernel's 168 VGPRs allow and cut the wave-steps
// that fall back to per-lane gathers from 18.6% to 6.9%: config-3 launch 501.0 -> 491.4 ms; 9 groups (11 blocks)
// 541 ms; 6 tile slots and 9 groups (12.4 KB) a further -0.9% (profiles/r06/ab/coop_groups_euler.txt)
#define MOPS_COOP_G 9
#endif
#ifndef MOPS_COOP_RETRY
#define MOPS_COOP_RETRY 64  // steps between regroup attempts of a wave in lane-normal mode (a power of two)
#endif
#ifndef MOPS_COOP_G_PR
#define MOPS_COOP_G_PR MOPS_COOP_G  // ... in the RK4 kernel (2 waves/SIMD by VGPRs: LDS to spare)
#endif
#ifndef MOPS_COOP_G_PRR
#define MOPS_COOP_G_PRR 16  // ... in the cooperative RK4 kernel behind the hand-off kernel: the waves handed over
                            // for more than MOPS_COOP_G_PR groups keep a tile (22 KB LDS, 6 blocks/CU for a tail
                            // kernel): config-3 RK4 launch 281.8 / 282.0 vs 283.5 / 284.5 ms at 9, 288 at 24
#endif
#ifndef MOPS_COOP_R_PR
#define MOPS_COOP_R_PR MOPS_COOP_R
#endif
#ifndef MOPS_TILE_SLOTS
#define MOPS_TILE_SLOTS 6  // polygon slots per tile group; 6: a wave with a heptagon lane gathers per lane, the
                           // others take 81 instead of 95 pieces per group (more groups in the same LDS)
#endif
static_assert(MOPS_TILE_SLOTS == 6 || MOPS_TILE_SLOTS == 7, "tile slots");
constexpr int kTileSlots = MOPS_TILE_SLOTS;
constexpr int kTilePoly = 2 * kTileSlots;  // 16-B pieces: the packed polygon slots {x, y, z, B_j}
constexpr int kCellNrm = 22;               // doubles per cell of mops_mesh::d_cnrm: 7 edge normals + pad
constexpr int kCellNrmPieces = kCellNrm / 2;  // ... as 11 pieces
constexpr int kTileNrm = (3 * kTileSlots + 1) / 2;  // the tile's normal pieces (7 slots: 11, 6 slots: 9)
constexpr int kTileRec = (kPairRec / 2) * kTileSlots;  // the slots' level-pair records of one field
#ifndef MOPS_TILE_E1
#define MOPS_TILE_E1 0  // the tile also holds each slot's edge vector X_{i+1} - X_i (mops_mesh::d_cedge): the
                        // Wachspress areas skip its 3 subtractions per slot (the same doubles, computed once per cell)
#endif
constexpr int kTileE1 = MOPS_TILE_E1 ? kTileNrm : 0;  // edge-vector pieces (laid out like the normals)
constexpr int kTileOffNrm = kTilePoly, kTileOffE1 = kTilePoly + kTileNrm, kTileOffRec = kTileOffE1 + kTileE1;
constexpr int kTilePieces = kTilePoly + kTileNrm + kTileE1 + 2 * kTileRec;  // 95 pieces = 1520 B per group (6 slots: 81)
constexpr int kTileHdr = 20;               // ints per group header: cell, nv, pad x2, front / back record index x 8
// Neighbour table (maxEdges <= 7 meshes, mops_mesh::d_nbr): per cell 112 B = 7 x 16 B -- the centre as three
// doubles, the 7 neighbour offsets q_k - c as floats, then the bitmask of the neighbours the walk considers.
// dev::nbr_stay answers the walk's "does c stay?" from it, exactly, in 7 VMEM instead of the walk's ~20.
#ifndef MOPS_NBR_TEST
#define MOPS_NBR_TEST 1
#endif
#ifndef MOPS_NBR_PAIR
#define MOPS_NBR_PAIR 0  // dev::nbr_stay re-arms the pair test (with MOPS_PAIR_TEST / MOPS_PAIR_TEST_P)
#endif
#ifndef MOPS_NBR_RK4
#define MOPS_NBR_RK4 0  // ... in the RK4 kernels too (measured: 6.64e9 vs 6.95e9 p-steps/s on the config-3 RK4 chain)
#endif
constexpr int kNbrQ = 7;                   // 16-B words per cell

}  // namespace

struct mops_mesh {
    int64_t C = 0, V = 0;
    int maxE = 0, L = 0;
    int maxv = 0;       // stencil capacity of the kernel instantiation (7, 12 or 20)
    int rec_ints = 0;   // ints per cell record
    int* d_cellrec = nullptr;    // [C][rec_ints]: nEdges | voc[maxv] | coc[maxv] (0-based, -1 none)
    double4* d_cxyz = nullptr;   // [C] (x,y,z,0)
    double4* d_vxyz = nullptr;   // [V]
    int* d_cov = nullptr;        // [V][3] cellsOnVertex 0-based, -1 = missing (boundary)
    double4* d_bary = nullptr;   // [V] barycentric weights in the cellsOnVertex centres (vertex_bary_kernel)
    // seed-location bucket index
    double bucket_h = 0.0, bucket_origin = 0.0;
    int origin_cell = -1;  // exact nearest centre to (0,0,0) (locate_kernel's tie rule)
    uint64_t* d_bkeys = nullptr;  // sorted bucket keys [C]
    int* d_bcells = nullptr;      // cell ids in key order [C]
    // bucket directory: open-addressing hash table (load <= 1/2) from a non-empty bucket's
    // key to its {first entry, entry count} in d_bkeys/d_bcells
    uint64_t* d_hkeys = nullptr;  // [H] key or ~0 (empty)
    int2* d_hval = nullptr;       // [H]
    uint32_t hmask = 0;           // H - 1
    uint32_t* d_cell_rank = nullptr;  // rank of each cell in the Morton order of the centres (particle locality order)
    int* d_rank_cell = nullptr;       // the inverse: the cell of each rank
    double2* d_cpolyr = nullptr;      // [2*7][C] d_cpoly's pieces by cell rank (maxv 7 meshes; MOPS_CPOLY_RANK)
    // [C][maxv] each cell's polygon in rotated slot order with its Wachspress weights' numerators:
    // slot j = {poly[j-1] (poly[-1] = poly[nv-1]), B_j = area(poly[j-1], poly[j], poly[j+1])}, zeros past nv
    double4* d_cpoly = nullptr;
    double* d_cnrm = nullptr;    // [C][kCellNrm] IsInMesh edge normals of the rotated polygon slots (maxv 7 meshes)
    double* d_cedge = nullptr;   // [C][kCellNrm] edge vectors X_{i+1} - X_i of the same slots (MOPS_TILE_E1)
    uint4* d_nbr = nullptr;      // [C][kNbrQ] neighbour table (cell_nbr_kernel, dev::nbr_stay; maxv 7 meshes)
    double* d_rloc2 = nullptr;       // [C] squared hinted-locate radius (locate_radius_kernel)
    double* d_ring = nullptr;        // [C] hinted-locate ring distance (locate_radius_kernel)
    // grow-only scratch for mops_order_particles (not re-entrant, like the reference's global app)
    mutable void* d_scratch = nullptr;
    mutable size_t scratch_bytes = 0;
    int64_t bytes = 0;
    std::vector<int> h_nv;  // nEdgesOnCell (host copy, for mops_mesh_set_edges' validation)
    // edges (mops_mesh_set_edges): the RBF reconstruction's per-cell stencil, solved once
    int64_t E = 0;
    int* d_eoc = nullptr;        // [C][7] edgesOnCell 0-based, -1 = none
    int2* d_coe = nullptr;       // [E] cellsOnEdge 0-based, -1 = none (the reference's SIZE_MAX)
    double4* d_exyz = nullptr;   // [E] edgeCoord
    double* d_rbf_coef = nullptr;  // [C][7][3] RBF coefficients (rbf_coef_kernel)
    int* d_rbf_slot = nullptr;     // [C][7] edge read by each slot, -1 = velocity 0
    // MOPS_VPERM: internal vertex i is the caller's vertex h_vold[i] (Morton order); every vertex-indexed array
    // (coordinates, cellsOnVertex, the derived fields and records) is internal, and the vertex ids in the cell
    // records are internal ids.  The vertex-array entry points map at the boundary (mops_field_create_derived,
    // mops_field_export: host rows; mops_cell_to_vertex_attr: d_vold).  Empty / NULL = identity.
    std::vector<int> h_vold;
    int* d_vold = nullptr;
    // the pathline launches' instantiation flag (coop_select_kernel), one per HIP stream: launches on
    // one stream run in order, so the next launch's selection never overwrites a flag a running
    // trajectory kernel still reads; allocated once per stream (no per-launch allocation)
    mutable std::mutex coop_mu;
    mutable std::vector<std::pair<hipStream_t, int*>> coop_flags;
};

struct mops_field {
    const mops_mesh* mesh = nullptr;
    int64_t V = 0;
    int L = 0;
    double* d_zt = nullptr;   // cellVertexZTop [V][L]
    double* d_vel = nullptr;  // cellVertexVelocity [V][L][3]
    double* d_w = nullptr;    // cellVertexVertVelocity [V][L+1]
    // [C] fast-path word (mono_kernel, read by dev::fast_ok): bit 31 = eligible, bits 20..26 = km,
    // the cell's decreasing prefix (every non-zero vertex column drops by >= 1e-6 m per level over
    // levels 0..km), bits 0..19 = which polygon slots are identically-zero columns (boundary
    // vertices, quirk Q10)
    uint32_t* d_mono = nullptr;
    int32_t* d_vmono = nullptr;  // [V] first level that breaks the vertex column's decrease (L = none)
    uint8_t* d_vzero = nullptr;  // [V] 1 = every level of the vertex column is 0 (boundary vertex)
    // level-pair records [V][L-1][kPairRec] doubles, record k-1 of vertex v =
    // {z_{k-1}, z_k, w_{k-1}, w_k, vel_{k-1} (3), vel_k (3)}: one 80-B,
    // 16-B-aligned read (5 x dwordx4) gives a vertex's whole contribution when
    // the particle sits in layer k
    double* d_pr = nullptr;
    // derivation intermediates (cell zTop [C][L], cell-centre xyz velocity [C][L][3]), kept
    // only by fields built from device arrays so mops_field_rebuild_device never allocates
    double* d_ztc = nullptr;
    double* d_velc = nullptr;
    // d_vel / d_w hold every value (fields uploaded as vertex arrays); false after the fused
    // derivation (pair_record_fused_kernel), which writes only the records, d_zt and w at level L:
    // mops_field_export then rebuilds d_vel / d_w from the records (records_to_vertex_kernel)
    bool vtx_full = true;
    int64_t bytes = 0;
};

// ===========================================================================
// device helpers -- every expression keeps the reference's evaluation order
// ===========================================================================
// ISA markers for instruction counting (tools/isa_marks.py; -DMOPS_ISA_MARKS builds only, never a
// product build): an assembly comment "@@MARK <id>" at the marked point
#if defined(MOPS_ISA_MARKS)
#define MOPS_MARK(id) asm volatile("; @@MARK %0" ::"i"(id))
#else
#define MOPS_MARK(id) do { } while (0)
#endif

namespace dev {

// Hand-off of LDS data between the lanes of one wave (the cooperative tile's headers and pieces): the
// wave's DS operations execute in issue order, so a wavefront-scope release/acquire pair -- no
// instructions, only an ordering the compiler must keep -- around a code-motion barrier suffices
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Zeros of records [k0, K) of one particle (records [K][6][stride]): what the reference's
// preallocated trajectory holds past a particle's death (the lambda returns, those points are
// never assigned) -- written once, at the death, instead of a memset of every record per run
__device__ __forceinline__ void clear_records(double* rec, int64_t stride, int64_t pid, int64_t k0, int64_t K) {
    for (int64_t k = k0; k < K; ++k) {
        double* rk = rec + k * 6 * stride + pid;
#pragma unroll
        for (int c = 0; c < 6; ++c) rk[c * stride] = 0.0;
    }
}

#if defined(MOPS_WAVE_STAMPS)
// Diagnostic builds only (tools/build_variant.sh -DMOPS_WAVE_STAMPS): 8 words per
// slot -- {start, end} in s_memrealtime ticks (100 MHz), the raw HW_ID / XCC_ID
// registers, then event counts: walks, cell loads after step 0, evaluations that
// missed the hinted fast bracket, zTop levels read by the brackets (low 32 bits)
// + bracket_scan calls (high 32).  Set with mops_debug_stamps; never in a product build.
__device__ unsigned long long* g_stamps;
__device__ long long g_stamps_cap;
__device__ __forceinline__ unsigned long long* stamp_slot() {
    const unsigned nblk = gridDim.x, b = blockIdx.x, xcd = b % 8u, q = nblk / 8u, r = nblk % 8u;
    const unsigned blk = (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + b / 8u;
    const long long slot = (long long)blk * blockDim.x + threadIdx.x;
    return (g_stamps && slot < g_stamps_cap) ? g_stamps + 8 * slot : nullptr;
}
#define MOPS_CNT(i, v) do { unsigned long long* _p = dev::stamp_slot(); if (_p) _p[i] += (v); } while (0)
#else
#define MOPS_CNT(i, v) do { } while (0)
#endif

// Ablation hooks for perf experiments only (tools/build_variant.sh -DMOPS_ABL_*):
// they break parity and are never set in a product build.
#if defined(MOPS_ABL_SQRT)
__device__ __forceinline__ double xsqrt(double x) { return x * __builtin_amdgcn_rsq(x); }
#else
// Correctly rounded sqrt, bit-identical to the compiler's sqrt(): for x in
// [2^-767, inf) its gfx950 expansion is exactly this rsq + Newton/Markstein
// sequence -- the input/output ldexp scaling (for x < 2^-767) and the +-0/+inf
// select around it are then identities, so they are skipped here.  Other x
// (0, tiny, inf, NaN, negative) take sqrt() itself.  Checked bitwise against
// sqrt() on the device and the host (mops_selftest_math, tests/test_gpu_parity.py).
__device__ __forceinline__ double sqrt_core(double x) {
    const double y = __builtin_amdgcn_rsq(x);
    double g = x * y;
    double h = y * 0.5;
    double r = __builtin_fma(-h, g, 0.5);
    g = __builtin_fma(g, r, g);
    h = __builtin_fma(h, r, h);
    double d = __builtin_fma(-g, g, x);
    g = __builtin_fma(d, h, g);
    d = __builtin_fma(-g, g, x);
    return __builtin_fma(d, h, g);
}
#ifndef MOPS_FAST_SQRT
#define MOPS_FAST_SQRT 1
#endif
#ifndef MOPS_SQRT_ONESIDED
#define MOPS_SQRT_ONESIDED 1  // measured: streamline Euler segment 27.0 -> 26.0 ms, RK4 86.5 -> 85.2 ms
#endif
__device__ __forceinline__ double xsqrt(double x) {
#if MOPS_FAST_SQRT && MOPS_SQRT_ONESIDED
    // the core result always, the library's only for the rare out-of-range x: a one-sided branch
    // (fewer exec-mask instructions than if/else)
    double r = sqrt_core(x);
    if (__builtin_expect(!(x >= 0x1p-767 && x < __builtin_huge_val()), 0)) r = sqrt(x);
    return r;
#else
#if MOPS_FAST_SQRT
    if (__builtin_expect(x >= 0x1p-767 && x < __builtin_huge_val(), 1)) return sqrt_core(x);
#endif
    return sqrt(x);
#endif
}
#endif

// An FP64 constant materialised in an SGPR pair at its point of use.  Plain
// literals are loop-invariant, so the compiler hoists them out of the step
// loop into VGPR pairs -- which at this kernel's register pressure are
// spilled to scratch and re-loaded from memory every step.  The s_mov_b32
// pair takes a loop-variant uniform input (`salt`, the step index) that it
// ignores, so it cannot be hoisted, yet (not volatile) it schedules freely.
__device__ __forceinline__ double kconst(unsigned hi, unsigned lo, unsigned salt) {
    unsigned h, l;
    asm("s_mov_b32 %0, %1" : "=s"(l) : "i"(lo), "s"(salt));
    asm("s_mov_b32 %0, %1" : "=s"(h) : "i"(hi), "s"(salt));
    return __hiloint2double((int)h, (int)l);
}
#define MOPS_K(bits) dev::kconst((unsigned)((bits) >> 32), (unsigned)((bits) & 0xffffffffULL), salt)

// a * b + k with k an SGPR-pair constant (MOPS_K), as one VOP3 v_fma_f64: the compiler's own
// choice is v_fmac_f64, whose tied accumulator needs k copied into a VGPR pair first (two
// v_mov_b32 per Horner step).  Same operation, same rounding.
#ifndef MOPS_SINCOS_VOP3
#define MOPS_SINCOS_VOP3 1
#endif
__device__ __forceinline__ double fma_k(double a, double b, double k) {
#if MOPS_SINCOS_VOP3
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "s"(k));
    return r;
#else
    return __builtin_fma(a, b, k);
#endif
}

// sin and cos of |x| < 0.78, bit-identical to the device library's sin(x) / cos(x):
// their gfx950 expansion reduces x by k = rint(|x| * 2/pi) with a Cody-Waite
// chain that, for k = 0, returns r = |x| and rr = +0 exactly, evaluates both
// kernel polynomials and selects by quadrant; sin takes the sign of x.  This is
// that k = 0 path with the same operations in the same order (the rr terms kept
// as literal +-0), skipping the reduction and the second polynomial of each
// call.  Checked bitwise against sin()/cos() (mops_selftest_math).
__device__ __forceinline__ void sincos_small(double x, double& s, double& c, unsigned salt) {
    const double r = fabs(x), rr = 0.0;
    const double x2 = r * r;
    const double h = x2 * 0.5;
    double t16 = __builtin_fma(MOPS_K(0xbda907db46cc5e42ULL), x2, MOPS_K(0x3e21eeb69037ab78ULL));
    const double t12 = 1.0 - h;
    double t18 = fma_k(x2, t16, MOPS_K(0xbe927e4fa17f65f6ULL));
    const double t14 = 1.0 - t12;
    t16 = fma_k(x2, t18, MOPS_K(0x3efa01a019f4ec90ULL));
    double t10 = t14 - h;
    t18 = fma_k(x2, t16, MOPS_K(0xbf56c16c16c16967ULL));
    const double x4 = x2 * x2;
    t16 = fma_k(x2, t18, MOPS_K(0x3fa5555555555555ULL));
    t10 = __builtin_fma(r, -rr, t10);
    t10 = __builtin_fma(x4, t16, t10);
    c = t12 + t10;
    double u12 = __builtin_fma(MOPS_K(0x3de5e0b2f9a43bb8ULL), x2, MOPS_K(0xbe5ae600b42fdfa7ULL));
    double u14 = fma_k(x2, u12, MOPS_K(0x3ec71de3796cde01ULL));
    u12 = fma_k(x2, u14, MOPS_K(0xbf2a01a019e83e5cULL));
    u14 = fma_k(x2, u12, MOPS_K(0x3f81111111110bb3ULL));
    u12 = r * -x2;
    double u16 = rr * 0.5;
    u16 = __builtin_fma(u12, u14, u16);
    double u4 = __builtin_fma(x2, u16, -rr);
    u4 = __builtin_fma(MOPS_K(0xbfc5555555555555ULL), u12, u4);
    const double sv = r - u4;
    s = __longlong_as_double(__double_as_longlong(sv) ^ (__double_as_longlong(x) & (long long)0x8000000000000000ULL));
}

// The library sin/cos for the rare |x| >= 0.78, out of line so that its
// constants are not hoisted into the step loop.
// (Returned by value: out-pointers to the caller's locals would pin them in
// scratch memory on every step, fast path included.)
__device__ __attribute__((noinline)) double2 sincos_lib(double x) {
    return make_double2(sin(x), cos(x));
}
#if defined(MOPS_ABL_DIV)
__device__ __forceinline__ double xdiv(double a, double b) { return a * __builtin_amdgcn_rcp(b); }
#else
__device__ __forceinline__ double xdiv(double a, double b) { return a / b; }
#endif

__device__ __forceinline__ double sq3(double x, double y, double z) { return x * x + y * y + z * z; }
__device__ __forceinline__ double len3(double x, double y, double z) { return xsqrt(sq3(x, y, z)); }

// q_j = a_j / b for the components of a vector and its length b = len3(a0, a1, a2)
// (b > 1e-12 checked by the caller), bit-identical to three `/`.  gfx950's
// correctly rounded a / b is div_scale(b), div_scale(a), rcp + two Newton steps
// on the scaled b, q = a*r, e = fma(-b, q, a), div_fmas(e, r, q), div_fixup.
// For b <= 2^300 and |a_j| >= 2^-700 no operand is scaled (b and 1/b normal,
// exponent(a) - exponent(b) <= 1 since |a_j| <= b (1 + 2^-52), a/b >=
// 2^-1000 normal, |a| >= 2^-969), so div_scale returns its input, div_fmas is
// a plain fma and div_fixup returns the finite nonzero quotient unchanged: the
// same operations on the same operands.  The reciprocal refinement depends on
// b alone, so it is done once for the three quotients (5 instead of 3 x 11
// instructions, one rcp instead of three).  Other operands (zero, tiny,
// NaN/inf) take `/`.  Checked bitwise against `/` (mops_selftest_math op 2).
#ifndef MOPS_FAST_DIV3
#define MOPS_FAST_DIV3 1
#endif
__device__ __forceinline__ void xdiv_norm3(double a0, double a1, double a2, double b, double& q0, double& q1,
                                           double& q2) {
#ifndef MOPS_DIV3_ONESIDED
#define MOPS_DIV3_ONESIDED 0
#endif
#if MOPS_FAST_DIV3 && !defined(MOPS_ABL_DIV)
    const bool fast = b <= 0x1p300 && fabs(a0) >= 0x1p-700 && fabs(a1) >= 0x1p-700 && fabs(a2) >= 0x1p-700;
#if MOPS_DIV3_ONESIDED
    if (true) {  // the fast quotients always; `/` replaces them for the rare operands outside the range
#else
    if (__builtin_expect(fast, 1)) {
#endif
        double r = __builtin_amdgcn_rcp(b);
        double e = __builtin_fma(-b, r, 1.0);
        r = __builtin_fma(r, e, r);
        e = __builtin_fma(-b, r, 1.0);
        r = __builtin_fma(r, e, r);
        double q = a0 * r;
        q0 = __builtin_fma(__builtin_fma(-b, q, a0), r, q);
        q = a1 * r;
        q1 = __builtin_fma(__builtin_fma(-b, q, a1), r, q);
        q = a2 * r;
        q2 = __builtin_fma(__builtin_fma(-b, q, a2), r, q);
#if MOPS_DIV3_ONESIDED
        if (__builtin_expect(!fast, 0)) { q0 = xdiv(a0, b); q1 = xdiv(a1, b); q2 = xdiv(a2, b); }
#endif
        return;
    }
#endif
    q0 = xdiv(a0, b); q1 = xdiv(a1, b); q2 = xdiv(a2, b);
}

// The reference's `length(v) < 1e-12` tests (MPASOVisualizerKernels.cpp:841-852)
// without the square root: correctly rounded sqrt is monotone, and the
// smallest double s with sqrt(s) >= 1e-12 is exactly the double 1e-24
// (0x1.357c299a88ea7p-80; tests/test_cpu_host.py::test_norm_threshold), so
// sqrt(s) < 1e-12  <=>  s < 1e-24 for every s >= 0, NaN and inf included.
constexpr double kNormTiny2 = 0x1.357c299a88ea7p-80;

// Interpolator::triangle_area (Interpolation.hpp:95-110)
__device__ __forceinline__ double tri_area(double ax, double ay, double az, double bx, double by, double bz,
                                           double cx, double cy, double cz) {
    const double e1x = bx - ax, e1y = by - ay, e1z = bz - az;
    const double e2x = cx - ax, e2y = cy - ay, e2z = cz - az;
    const double px = e1y * e2z - e1z * e2y;
    const double py = e1z * e2x - e1x * e2z;
    const double pz = e1x * e2y - e1y * e2x;
    return xsqrt(px * px + py * py + pz * pz) / 2.0;
}

// Wachspress without the two halvings (round 6, MOPS_WACH_X4): the reference's w_i = B_i / (A_i A_{i+1}) with
// A = R / 2, R = sqrt(|cross|^2).  Halving is exact here, and so is scaling a product by 1/4 before rounding: with
// mesh vertices at Earth radius (< 2^23 m) every edge difference is a multiple of 2^-30, every cross-product
// component a multiple of 2^-60, so R is 0 or >= 2^-60 and R_i R_{i+1} is 0 or >= 2^-120 -- far from the
// subnormal range, and far below overflow.  So fl(A_i A_{i+1}) = fl(R_i R_{i+1}) / 4 and fl(B_i / fl(A_i A_{i+1})) = fl(4 B_i / fl(R_i R_{i+1}))
// with 4 B_i exact: the same double, inf (R = 0) and NaN included, from 4 B_i stored per cell (cell_poly_kernel,
// load_cell) and R_i = tri_area_x2: 6 FP64 multiplies fewer per evaluation.
#ifndef MOPS_WACH_X4
#define MOPS_WACH_X4 1
#endif
__device__ __forceinline__ double tri_area_x2(double ax, double ay, double az, double bx, double by, double bz,
                                              double cx, double cy, double cz) {
    const double e1x = bx - ax, e1y = by - ay, e1z = bz - az;
    const double e2x = cx - ax, e2y = cy - ay, e2z = cz - az;
    const double px = e1y * e2z - e1z * e2y;
    const double py = e1z * e2x - e1x * e2z;
    const double pz = e1x * e2y - e1y * e2x;
    return xsqrt(px * px + py * py + pz * pz);
}
// ... with the edge vector e1 = b - a given (the same doubles: MOPS_TILE_E1 stores b - a per cell)
__device__ __forceinline__ double tri_area_x2_e(double ax, double ay, double az, double e1x, double e1y, double e1z,
                                                double cx, double cy, double cz) {
    const double e2x = cx - ax, e2y = cy - ay, e2z = cz - az;
    const double px = e1y * e2z - e1z * e2y;
    const double py = e1z * e2x - e1x * e2z;
    const double pz = e1x * e2y - e1y * e2x;
    return xsqrt(px * px + py * py + pz * pz);
}
// the per-cell Wachspress numerator as the weights read it: B_i, or 4 B_i (exact) with MOPS_WACH_X4
__device__ __forceinline__ double wach_numerator(double B) { return MOPS_WACH_X4 ? 4.0 * B : B; }

// TBBKernel::CalcPositionAfterRotation (TBBKernel.h:177-206)
__device__ __forceinline__ void rotate(unsigned salt, double px, double py, double pz, double ax, double ay, double az, double th,
                                       double& rx, double& ry, double& rz) {
#if defined(MOPS_ABL_TRIG)
    const double c = 1.0 - 0.5 * th * th, s = th;
#else
    double c, s;
#ifndef MOPS_FAST_TRIG
#define MOPS_FAST_TRIG 1
#endif
#ifndef MOPS_TRIG_ONESIDED
#define MOPS_TRIG_ONESIDED 0
#endif
#if MOPS_TRIG_ONESIDED
    sincos_small(th, s, c, salt);  // always; the library's values replace it for the rare |th| >= 0.78
    if (!MOPS_FAST_TRIG || __builtin_expect(!(fabs(th) < 0.78), 0)) {
        const double2 sc = sincos_lib(th);
        s = sc.x;
        c = sc.y;
    }
#else
    if (MOPS_FAST_TRIG && __builtin_expect(fabs(th) < 0.78, 1)) {
        sincos_small(th, s, c, salt);
    } else {
        const double2 sc = sincos_lib(th);
        s = sc.x;
        c = sc.y;
    }
#endif
#endif
    const double al = len3(ax, ay, az);
    if (al <= 1e-12) { rx = px; ry = py; rz = pz; return; }
    double ux, uy, uz;
    xdiv_norm3(ax, ay, az, al, ux, uy, uz);
    rx = (c + ux * ux * (1.0 - c)) * px + (ux * uy * (1.0 - c) - uz * s) * py + (ux * uz * (1.0 - c) + uy * s) * pz;
    ry = (uy * ux * (1.0 - c) + uz * s) * px + (c + uy * uy * (1.0 - c)) * py + (uy * uz * (1.0 - c) - ux * s) * pz;
    rz = (uz * ux * (1.0 - c) - uy * s) * px + (uz * uy * (1.0 - c) + ux * s) * py + (c + uz * uz * (1.0 - c)) * pz;
}

// advect_on_sphere lambda (MPASOVisualizerKernels.cpp:729-738)
__device__ __forceinline__ void advect(unsigned salt, double px, double py, double pz, double vx, double vy, double vz, double dt,
                                       double& ox, double& oy, double& oz) {
    const double rr = len3(px, py, pz), sp = len3(vx, vy, vz);
    if (rr < 1e-12 || sp < 1e-12) { ox = px; oy = py; oz = pz; return; }
    const double ax = py * vz - pz * vy, ay = pz * vx - px * vz, az = px * vy - py * vx;
    const double th = (sp * dt) / rr;
    rotate(salt, px, py, pz, ax, ay, az, th, ox, oy, oz);
}

__device__ __forceinline__ double dmax(double a, double b) { return (a < b) ? b : a; }  // std::max
__device__ __forceinline__ double dmin(double a, double b) { return (b < a) ? b : a; }  // std::min
__device__ __forceinline__ double dclamp(double v, double lo, double hi) { return (v < lo) ? lo : (hi < v) ? hi : v; }

// Per-mode polygon cache (swept on MI355X): 1 = vertex xyz + B_i
// live in registers while the particle stays in its cell; 0 = re-read per
// evaluation (L1-resident), which frees ~56 VGPRs for the heavier modes.
#ifndef MOPS_RC_SE
#define MOPS_RC_SE 1
#endif
#ifndef MOPS_RC_SR
#define MOPS_RC_SR 1
#endif
#ifndef MOPS_RC_PE
#define MOPS_RC_PE 0
#endif
#ifndef MOPS_RC_PR
#define MOPS_RC_PR 0
#endif
#ifndef MOPS_RC_PE_PLAIN
#define MOPS_RC_PE_PLAIN 0
#endif
// modes without the register polygon: read a slot from the per-cell packed polygon (one 32-B
// {x, y, z, B_j}, mops_mesh::d_cpoly) rather than the vertex array + B_j (1 = packed)
#ifndef MOPS_CPOLY
#define MOPS_CPOLY 1
#endif
// ... and (MAXV 7) read it piece-major in the cells' Morton-rank order, mops_mesh::d_cpolyr [14][C]: the lanes of a
// wave sit in consecutive-rank cells (the particles' locality order), so one polygon-piece gather touches a few
// 128-B lines instead of one per cell (the TD spends a cycle per line)
#ifndef MOPS_CPOLY_RANK
#define MOPS_CPOLY_RANK 1
#endif

// Per-cell stencil cached in registers while the particle stays in the cell.
template <int MAXV>
struct Cell {
    int id;
    int nv;
    uint32_t mono0, mono1;  // fast-path words of the cell for the front / back field (mops_field::d_mono)
    double cx, cy, cz;  // "stay" anchor: the cell centre, or the position of the last walk that kept the cell
    double rs2;         // squared stay radius around the anchor (see dev::walk)
    int vid[MAXV];
    int vlast;          // vid[nv-1]: slot 0 of the rotated polygon
    int V;              // vertex count (index of the all-zero level-pair record is V*(L-1))
    bool rc;            // compile-time constant per kernel (load_cell<MAXV, RC>): which members below are live
    // polygon positions in "rotated" order: x[0] = poly[nv-1], x[j] = poly[j-1] (1 <= j < nv), so
    // that edge k (poly[k-1], poly[k]) and the reference's running triangle A_k = area(poly[k-1],
    // poly[k], p) are the slot pair (k, k+1), wrapping to slot 0 only at k = nv-1
    double x[MAXV], y[MAXV], z[MAXV];
    double B[MAXV];  // Wachspress B_i = area(poly[i-1], poly[i], poly[i+1]) (depends on the polygon only)
    bool lds_n;         // nrm below is live: constant per kernel, or the cooperative kernel's per-wave mode
    // lds_n: IsInMesh edge normals n_i = X_i x X_{i+1} (slot pairs as in dev::weights), computed
    // by load_cell into this lane's LDS column: component j of slot i at nrm[(3 * i + j) * kTrajBlock]
    double* nrm;
    // pair test (dev::walk): the bisector of c and its nearest neighbour at the last anchor, valid
    // in a second, larger ball around it -- {n.x, n.y, n.z, k, rb2} at pr2[j * kTrajBlock] (LDS);
    // rb2 < 0 = none (load_cell)
    double* pr2;
    float* rb2;      // MOPS_LDS_COMPACT: the pair test's rb2 (else pr2[4 * kTrajBlock])
    const double4* __restrict__ vxyz;   // rc == false: polygon re-read per evaluation (L1-resident)
    const double4* __restrict__ cpoly;  // rc == false: per-cell rotated polygon + B_i [C][MAXV] (cell_poly_kernel)
    const double2* __restrict__ cpolyr;  // MOPS_CPOLY_RANK: the same, piece-major by cell rank [2 MAXV][C]
    const uint32_t* __restrict__ crank;  // mops_mesh::d_cell_rank
    uint32_t rank, C;                    // this cell's rank (load_cell), the cell count
};

// NRMC (the cooperative kernel): the lane's normals, when it keeps them (c.lds_n, a wave-uniform
// runtime mode there), are copied from the per-cell array mops_mesh::d_cnrm -- the same products
template <int MAXV, bool RC, bool NRM, bool PT, bool NRMC = false>
__device__ __forceinline__ void load_cell(Cell<MAXV>& c, int cell, const int* __restrict__ cellrec,
                                          const double4* __restrict__ vxyz, const uint32_t* __restrict__ mono0,
                                          const uint32_t* __restrict__ mono1, const double4* __restrict__ cxyz,
                                          const double4* __restrict__ cpoly, const double* __restrict__ cnrm = nullptr) {
    c.mono0 = mono0[cell];
    c.mono1 = mono1[cell];
    {
        const double4 q = cxyz[cell];
        c.cx = q.x; c.cy = q.y; c.cz = q.z; c.rs2 = q.w;
    }
    if constexpr (PT) {  // no pair test before a walk in c
        if (MOPS_LDS_COMPACT) *c.rb2 = -1.0f;
        else c.pr2[4 * kTrajBlock] = -1.0;
    }
    constexpr int REC = ((1 + 2 * MAXV) + 3) / 4 * 4;
    const int* r = cellrec + (int64_t)cell * REC;
    int buf[REC];
#pragma unroll
    for (int q = 0; q < REC / 4; ++q) {
        const int4 v = reinterpret_cast<const int4*>(r)[q];
        buf[4 * q] = v.x; buf[4 * q + 1] = v.y; buf[4 * q + 2] = v.z; buf[4 * q + 3] = v.w;
    }
    c.id = cell;
    c.nv = buf[0];
    const int nv = c.nv;
    c.rc = RC;
#pragma unroll
    for (int k = 0; k < MAXV; ++k) c.vid[k] = buf[1 + k];
    c.vlast = 0;
#pragma unroll
    for (int k = 0; k < MAXV; ++k)
        if (k == nv - 1) c.vlast = c.vid[k];
    if constexpr (!RC) {
        c.vxyz = vxyz;
        c.cpoly = cpoly;
        if constexpr (MOPS_CPOLY_RANK && MAXV == 7) c.rank = c.crank[cell];
    }
    if constexpr (NRMC) {
        if (c.lds_n) {
            const double* src = cnrm + (int64_t)cell * kCellNrm;
#pragma unroll
            for (int k = 0; k < 3 * kNrmSlots(MAXV); ++k) c.nrm[k * kTrajBlock] = src[k];
        }
    } else if constexpr (RC || NRM) {
        double px[MAXV], py[MAXV], pz[MAXV];  // natural order
#pragma unroll
        for (int k = 0; k < MAXV; ++k) {
            if (k < nv) {
                const double4 p = vxyz[c.vid[k]];
                px[k] = p.x; py[k] = p.y; pz[k] = p.z;
            } else {
                px[k] = 0.0; py[k] = 0.0; pz[k] = 0.0;
            }
        }
        double lx = 0, ly = 0, lz = 0;  // poly[nv-1]
#pragma unroll
        for (int k = 0; k < MAXV; ++k)
            if (k == nv - 1) { lx = px[k]; ly = py[k]; lz = pz[k]; }
        // edge normals: rotated slot pair i (see Cell) is (poly[i-1], poly[i]), poly[-1] = poly[nv-1]
#pragma unroll
        for (int i = 0; i < MAXV; ++i) {
            if (NRM && i < nv && i < kNrmSlots(MAXV)) {
                const double qx = (i == 0) ? lx : px[(i + MAXV - 1) % MAXV];
                const double qy = (i == 0) ? ly : py[(i + MAXV - 1) % MAXV];
                const double qz = (i == 0) ? lz : pz[(i + MAXV - 1) % MAXV];
                c.nrm[(3 * i + 0) * kTrajBlock] = qy * pz[i] - qz * py[i];
                c.nrm[(3 * i + 1) * kTrajBlock] = qz * px[i] - qx * pz[i];
                c.nrm[(3 * i + 2) * kTrajBlock] = qx * py[i] - qy * px[i];
            }
        }
        if constexpr (RC) {
#pragma unroll
            for (int i = 0; i < MAXV; ++i) {
                if (i < nv) {
                    const double qx = (i == 0) ? lx : px[(i + MAXV - 1) % MAXV];
                    const double qy = (i == 0) ? ly : py[(i + MAXV - 1) % MAXV];
                    const double qz = (i == 0) ? lz : pz[(i + MAXV - 1) % MAXV];
                    const bool wrap = (i + 1 >= nv);
                    const double nx = wrap ? px[0] : px[(i + 1) % MAXV];
                    const double ny = wrap ? py[0] : py[(i + 1) % MAXV];
                    const double nz = wrap ? pz[0] : pz[(i + 1) % MAXV];
                    c.B[i] = wach_numerator(tri_area(qx, qy, qz, px[i], py[i], pz[i], nx, ny, nz));
                } else {
                    c.B[i] = 0.0;
                }
            }
            c.x[0] = lx; c.y[0] = ly; c.z[0] = lz;
#pragma unroll
            for (int j = 1; j < MAXV; ++j) { c.x[j] = px[j - 1]; c.y[j] = py[j - 1]; c.z[j] = pz[j - 1]; }
        }
    }
}

// The cell's vertex count as the evaluation sees it: NV > 0 is a compile-time
// count the caller has checked for every lane of the wave (eval_at), so the
// per-slot `v < nv` masks and the polygon's wrap-around selects fold away;
// NV = 0 reads it from the cell.
#ifndef MOPS_HEX
#define MOPS_HEX 1  // NV = 6 instantiation for all-hexagon waves
#endif
// ... and for the level-pair sums: pathline yes (measured -2%, PE/PR); streamline no --
// without the per-vertex branch its scheduler spills (register-cached polygon), 2.4x slower
#ifndef MOPS_HEX_PAIRS
#define MOPS_HEX_PAIRS 0
#endif
#ifndef MOPS_HEX_PAIRS_P
#define MOPS_HEX_PAIRS_P 1
#endif
template <int NV, int MAXV>
__device__ __forceinline__ int nverts(const Cell<MAXV>& c) { return NV > 0 ? NV : c.nv; }

// guards + TBBKernel::IsInMesh + Interpolator::CalcPolygonWachspress
// (MPASOVisualizerKernels.cpp:744-770, TBBKernel.h:21-54, Interpolation.hpp:137-165)
template <int MAXV, int NV, bool COOP = false, bool BAR = true>
__device__ __forceinline__ bool weights(const Cell<MAXV>& c, int L, int V, double px, double py, double pz,
                                        double* w, const double4* tpoly = nullptr) {
    if (c.id < 0 || L <= 1 || L > kMaxLevels) return false;
    const int nv = nverts<NV>(c);
    if (nv <= 0 || nv > kMaxVertex) return false;
    if (!isfinite(px) || !isfinite(py) || !isfinite(pz)) return false;
    // rotated slots (see Cell): X[0] = poly[nv-1], X[j] = poly[j-1]
    double X[MAXV], Y[MAXV], Z[MAXV], BB[MAXV];
#pragma unroll
    for (int j = 0; j < MAXV; ++j) {
        if (c.rc) {
            X[j] = c.x[j]; Y[j] = c.y[j]; Z[j] = c.z[j]; BB[j] = c.B[j];
        } else {
            if (j < nv) {
#if MOPS_CPOLY
                // one 32-B slot {x, y, z, B_j} of the cell's packed polygon: 2 VMEM instead of 3; in a
                // cooperative wave (coop, wave-uniform) the same slot from the wave's LDS tile
                double4 q;
                if constexpr (COOP) {
                    q = tpoly[j];
                } else if constexpr (MOPS_CPOLY_RANK && MAXV == 7) {
                    const double2 lo = c.cpolyr[(uint32_t)(2 * j) * c.C + c.rank];
                    const double2 hi = c.cpolyr[(uint32_t)(2 * j + 1) * c.C + c.rank];
                    q = make_double4(lo.x, lo.y, hi.x, hi.y);
                } else {
                    q = c.cpoly[(int64_t)c.id * MAXV + j];
                }
                X[j] = q.x; Y[j] = q.y; Z[j] = q.z; BB[j] = q.w;
#else
                const double4 q = c.vxyz[j == 0 ? c.vlast : c.vid[(j + MAXV - 1) % MAXV]];
                X[j] = q.x; Y[j] = q.y; Z[j] = q.z;
                BB[j] = c.cpoly[(int64_t)c.id * MAXV + j].w;
#endif
            } else {
                X[j] = 0.0; Y[j] = 0.0; Z[j] = 0.0; BB[j] = 0.0;
            }
        }
    }
    // one pass over the slot pairs (X[i], X[i+1]) -- (X[nv-1], X[0]) at the wrap -- which are both the
    // polygon's edges (poly[i-1], poly[i]) for IsInMesh (a conjunction of side-effect-free tests, so the
    // order of the edges is immaterial) and the arguments of A_i = area(poly[i-1], poly[i], p)
    // (Interpolation.hpp:137-165: A_0 = area(poly[N-1], poly[0], p), A_{i+1} = area(poly[i], poly[i+1], p));
    // A_i is kept in w[i] until the weights are formed
    MOPS_MARK(200 + NV);
    bool inside = true;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
        if (i < nv) {
            const bool wrap = (i + 1 >= nv);
            const double bx = wrap ? X[0] : X[(i + 1) % MAXV];
            const double by = wrap ? Y[0] : Y[(i + 1) % MAXV];
            const double bz = wrap ? Z[0] : Z[(i + 1) % MAXV];
            double nx, ny, nz;  // the edge normal X_i x X_{i+1}: cached per cell (load_cell) or computed
            if constexpr (COOP) {  // the tile's copy of the cell's normals (mops_mesh::d_cnrm)
                const double* tn = reinterpret_cast<const double*>(tpoly + kTilePoly / 2);
                nx = tn[3 * i]; ny = tn[3 * i + 1]; nz = tn[3 * i + 2];
            } else if (c.lds_n && i < kNrmSlots(MAXV)) {
                nx = c.nrm[(3 * i + 0) * kTrajBlock]; ny = c.nrm[(3 * i + 1) * kTrajBlock]; nz = c.nrm[(3 * i + 2) * kTrajBlock];
            } else {
                nx = Y[i] * bz - Z[i] * by;
                ny = Z[i] * bx - X[i] * bz;
                nz = X[i] * by - Y[i] * bx;
            }
            inside = inside & !(nx * px + ny * py + nz * pz < 0.0);  // no short circuit: straight-line code
            if constexpr (COOP && MOPS_TILE_E1 && MOPS_WACH_X4) {  // the tile's b - a of this slot
                const double* te = reinterpret_cast<const double*>(tpoly) + 2 * kTileOffE1;
                w[i] = tri_area_x2_e(X[i], Y[i], Z[i], te[3 * i], te[3 * i + 1], te[3 * i + 2], px, py, pz);
            } else {
                w[i] = MOPS_WACH_X4 ? tri_area_x2(X[i], Y[i], Z[i], bx, by, bz, px, py, pz)
                                    : tri_area(X[i], Y[i], Z[i], bx, by, bz, px, py, pz);
            }
            if constexpr (NV > 0 && BAR) __builtin_amdgcn_sched_barrier(0);  // one slot at a time (register pressure)
        } else {
            w[i] = 0.0;
        }
    }
    MOPS_MARK(210 + NV);
    if (!inside) return false;
    // (the reference also range-checks the vertex ids in its zTop loop, :776-779; mops_mesh_create
    // rejects a mesh with an out-of-range active verticesOnCell entry, so that test always passes)
    // w_i = B_i / (A_i * A_{i+1}), A_nv = A_0, summed in vertex order
    const double A0 = w[0];
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
        if (i < nv) {
            const double An = (i + 1 >= nv) ? A0 : w[(i + 1) % MAXV];
            w[i] = xdiv(BB[i], (w[i] * An));
            sum += w[i];
        }
    }
    const double recp = xdiv(1.0, sum);
#pragma unroll
    for (int i = 0; i < MAXV; ++i)
        if (i < nv) w[i] *= recp;
    MOPS_MARK(220 + NV);
    return true;
}

// one interpolated zTop level:  z = sum_v w_v * zTopV[v*L + k]  (v in order)
template <int MAXV>
__device__ __forceinline__ double col(const Cell<MAXV>& c, const double* w, const double* __restrict__ zt, int L,
                                      int k) {
    MOPS_CNT(7, 1);
    double acc = 0.0;
#pragma unroll
    for (int v = 0; v < MAXV; ++v)
        if (v < c.nv) acc += w[v] * zt[(int64_t)c.vid[v] * L + k];
    return acc;
}

// Layer bracket over the interpolated, monotone-fixed zTop column
// (streamline :772-822, pathline :1156-1218) without materialising it.
//
// The fixed-up column z' (z'_k = z_k > z'_{k-1} ? z'_{k-1} - 1e-9 : z_k) is
// non-increasing, so P(k) = d <= z'_{k-1}+eps is true exactly for k <= b and
// Q(k) = d >= z'_k-eps exactly for k >= a (rounding is monotone).  Every
// comparison the reference's binary search (streamline) or linear scan
// (pathline) makes is P or Q, so its result is a function of (a, b) alone:
// the scan stops at the first level where both are known.  If a exists the
// reference's "below the bottom" test is provably false (z'_{L-1} <= z'_a).
// Returns the layer (or -1 = fail) and z'_layer, z'_{layer-1}.
template <int MAXV, bool PATH>
__device__ __forceinline__ int bracket_scan(const Cell<MAXV>& c, const double* w, const double* __restrict__ zt,
                                            int L, double d, double& zdn, double& zup) {
    const double eps = 1e-8;
    const double z0 = col<MAXV>(c, w, zt, L, 0);
    double z1 = col<MAXV>(c, w, zt, L, 1);
    MOPS_CNT(7, 1ull << 32);
    if (z1 > z0) z1 = z0 - 1e-9;
    if (d > z0 + eps) {  // above the surface (PATH: reference layer 0 reads z[-1])
        zdn = z1; zup = z0;
        return 1;
    }
    int a = -1, b = -1;
    double za = 0, za_m1 = 0, zb = 0, zb_m1 = 0;
    double zpp = z0, zp = z0;  // z'_{k-2}, z'_{k-1}
    for (int k = 1; k < L; ++k) {
        double zk;
        if (k == 1) {
            zk = z1;
        } else {
            zk = col<MAXV>(c, w, zt, L, k);
            if (zk > zp) zk = zp - 1e-9;
        }
        const bool P = d <= zp + eps;
        const bool Q = d >= zk - eps;
        if (a < 0 && Q) { a = k; za = zk; za_m1 = zp; }
        if (b < 0 && !P) { b = k - 1; zb = zp; zb_m1 = zpp; }
        zpp = zp;
        zp = zk;
        if (a >= 0 && b >= 0) break;
    }
    if (b < 0) { b = L - 1; zb = zp; zb_m1 = zpp; }
    if (a < 0) {  // scanned the whole column: zp = z'_{L-1}, zpp = z'_{L-2}
        if (d < zp - eps) { zdn = zp; zup = zpp; return L - 1; }
    }
    int layer;
    if (PATH) {
        if (a < 0 || a > b) return -1;  // linear scan found nothing
        layer = a;
    } else {
        const int aa = (a < 0) ? L : a;
        int lo = 1, hi = L - 1, ans = 1;
        while (lo <= hi) {
            const int mid = (lo + hi) >> 1;
            if (mid >= aa && mid <= b) { ans = mid; break; }
            if (mid > b) hi = mid - 1; else lo = mid + 1;
        }
        layer = ans;
    }
    if (layer == a) { zdn = za; zup = za_m1; return layer; }
    if (layer == b && b >= 2) { zdn = zb; zup = zb_m1; return layer; }
    if (layer == 1) { zdn = z1; zup = z0; return 1; }
    // rare (a level thinner than 2e-8 inside the bracket): recompute the chain
    double p = z0, q = z0;
    for (int k = 1; k <= layer; ++k) {
        double zk = col<MAXV>(c, w, zt, L, k);
        if (zk > p) zk = p - 1e-9;
        q = p;
        p = zk;
    }
    zdn = p; zup = q;
    return layer;
}

// Fast, exact bracket for a particle whose interpolated column is provably
// strictly decreasing over its first km + 1 levels (fast_ok: km = the cell's
// decreasing prefix, every non-zero vertex column drops by >= 1e-6 m per
// level there): the reference's fix-up never fires on levels 1..km, so z'_k
// = z_k there, computable level by level, and the bracket predicates are
// monotone in the level everywhere (the fixed column is non-increasing by
// construction).  a and b (see bracket_scan) are then found by walking from
// the particle's previous layer (`hint`, clamped to km); typically two levels
// plus the surface level are read instead of the whole column.  Any hint gives
// the same result.  Below the prefix the fix-up may fire, so a walk towards the
// bottom continues the reference's recurrence z'_k = z_k > z'_{k-1} ? z'_{k-1}
// - 1e-9 : z_k from z'_{k-1} (exact: the chain starts inside the prefix, where
// z' = z).  That keeps a partial-bottom column (flat zero-thickness layers under
// the local bottom, km < L-1) off the whole-column scan for a particle sitting
// below its bottom.  A NaN below the prefix (the column is no longer
// non-increasing there) returns -2 and the caller runs bracket_scan, as does a
// binary-search layer strictly inside (a, b) below the prefix.
template <int MAXV, bool PATH>
__device__ __forceinline__ int bracket_mono(const Cell<MAXV>& c, const double* w, const double* __restrict__ zt,
                                            int L, int km, double d, int& hint, double& zdn, double& zup) {
    const double eps = 1e-8;
    int h = (hint > km) ? km : hint;
    const bool hint_ok = (h >= 1);
    if (!hint_ok) h = 1;
    // one batch of independent loads: z_0, z_{h-1}, z_h (per-level sums keep
    // the reference's vertex order)
    double z0 = 0.0, zhm1 = 0.0, zh = 0.0;
#pragma unroll
    for (int v = 0; v < MAXV; ++v) {
        if (v < c.nv) {
            const double* q = zt + (int64_t)c.vid[v] * L;
            const double q0 = q[0], q1 = q[h - 1], q2 = q[h];
            z0 += w[v] * q0;
            zhm1 += w[v] * q1;
            zh += w[v] * q2;
        }
    }
    if (d > z0 + eps) {  // above the surface (PATH: see DESIGN.md Q4)
        zdn = (h == 1) ? zh : ((h == 2) ? zhm1 : col<MAXV>(c, w, zt, L, 1));
        zup = z0; hint = 1;
        return 1;
    }
    if (!hint_ok) {  // no hint: lower_bound of Q over [1, km] by bisection
        int lo = 1, hi = km + 1;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (d >= col<MAXV>(c, w, zt, L, mid) - eps) hi = mid; else lo = mid + 1;
        }
        h = (lo <= km) ? lo : km;  // lo > km: a lies below the prefix, walk down from km
        zh = col<MAXV>(c, w, zt, L, h);
        zhm1 = (h == 1) ? z0 : col<MAXV>(c, w, zt, L, h - 1);
    }
    int a;
    double za, zam1;  // z_a, z_{a-1}
    if (d >= zh - eps) {  // a <= h: walk towards the surface
        int k = h;
        double zk = zh;
        double zkm1 = zhm1;
        while (k > 1 && d >= zkm1 - eps) {
            --k;
            zk = zkm1;
            zkm1 = (k == 1) ? z0 : col<MAXV>(c, w, zt, L, k - 1);
        }
        a = k; za = zk; zam1 = zkm1;
    } else {  // a > h: walk towards the bottom
        int k = h;
        double zk = zh, zprev = zh;
        bool found = false;
        while (k < L - 1) {
            ++k;
            zprev = zk;
            zk = col<MAXV>(c, w, zt, L, k);
            if (k > km) {  // the reference's fix-up (a no-op inside the prefix)
                if (isnan(zk)) return -2;
                if (zk > zprev) zk = zprev - 1e-9;
            }
            if (d >= zk - eps) { found = true; break; }
        }
        if (!found) {  // Q(L-1) false  <=>  d < z'_{L-1} - eps: the "below the bottom" branch
            const double zlm1 = (k == h) ? zhm1 : zprev;
            zdn = zk; zup = zlm1; hint = L - 1;
            return L - 1;
        }
        a = k; za = zk; zam1 = zprev;
    }
    // b = last k with P(k) = d <= z_{k-1} + eps; P(a) holds (a == 1: not above
    // the surface; a > 1: !Q(a-1))
    int b = a;
    double zb = za, zbm1 = zam1;
    while (b < L - 1 && d <= zb + eps) {
        double zn = col<MAXV>(c, w, zt, L, b + 1);
        if (b + 1 > km) {
            if (isnan(zn)) return -2;
            if (zn > zb) zn = zb - 1e-9;
        }
        zbm1 = zb; zb = zn; ++b;
    }
    int layer;
    if (PATH) {
        layer = a;  // linear scan: first k with P && Q
    } else {        // the reference's binary search, driven by (a, b)
        int lo = 1, hi = L - 1, ans = 1;
        while (lo <= hi) {
            const int mid = (lo + hi) >> 1;
            if (mid >= a && mid <= b) { ans = mid; break; }
            if (mid > b) hi = mid - 1; else lo = mid + 1;
        }
        layer = ans;
    }
    if (layer == a) { zdn = za; zup = zam1; }
    else if (layer == b) { zdn = zb; zup = zbm1; }
    else if (layer > km) return -2;  // strictly inside (a, b) below the prefix: needs the whole chain
    else { zdn = col<MAXV>(c, w, zt, L, layer); zup = col<MAXV>(c, w, zt, L, layer - 1); }
    hint = layer;
    return layer;
}

// One-hop nearest-centre walk (TBBKernel::GetCellNeighborsIdx, TBBKernel.h:74-101,
// and the relocation loop, MPASOVisualizerKernels.cpp:902-922): candidates are
// cellsOnCell[c][0..nv-1] then c itself, entries outside [0, C) skipped, and
// the first candidate with the smallest Euclidean distance wins (strict <).
// All neighbour ids and centres are fetched in one batch (the reference's loop
// order would serialise 2 round trips per candidate), and the argmin runs on
// squared distances: correctly rounded sqrt is monotone, so the smallest
// distance is sqrt(min s), and a later candidate ties it only if its s is
// within a few ulps of min s -- only then is its sqrt taken and compared.  A
// candidate whose distance is inf or NaN never beats the reference's initial
// DBL_MAX, so only finite s take part.
//
// Stay anchor.  When the walk keeps c, every neighbour is farther than c by
// the gap g = sqrt(s_2nd) - sqrt(s_c) (computed; its error, like that of every
// computed distance here, is < 1e-7 m at Earth radius).  Moving the particle
// by delta changes each distance by at most delta, so for |p - p0| < (g -
// 0.01 m) / 2 every neighbour stays farther than c by more than rounding and
// the reference's argmin keeps c with the same candidate list: the caller
// skips the walk inside that ball (anchor p0 = this position).  load_cell
// sets the anchor to the cell centre with rs = (min_nb |c_nb - c|)/2 - 1 m,
// the same argument at p0 = c.  A walk that changes cell leaves the anchor of
// the new cell's load_cell.
//
// Pair test (MOPS_PAIR_TEST).  Near an edge of c the stay ball is small (g is the gap to the
// neighbour across that edge), so a particle drifting along the edge walked every few steps --
// the walk's gathers and their dependent round trips cost ~14% of a config-2 step (measured by
// running every walk twice).  The walk that keeps c therefore also records, for its anchor p0, the
// gap g2 of the second-nearest distinct neighbour and the bisector of c and the nearest one, nb1:
// f(p) = |p - c1|^2 - |p - c|^2 = n.p + k, n = 2 (c - c1), k = |c1|^2 - |c|^2.  Inside the ball
// |p - p0| < (g2 - 0.01 m) / 2 every neighbour but nb1 stays farther than c by more than rounding
// (same argument as above), so the reference's argmin is c or nb1; and there d_1 + d_c <= D =
// 2 rb + d_c(p0) + d_1(p0), so f(p) > 0.01 D means d_1 - d_c > 0.01 m, far above the < 1e-7 m
// error of a computed distance, i.e. c stays the unique minimum.  The computed f errs by < 1e-13
// (|c|^2 + |c1|^2 + |p0|^2 + rb^2) (a few hundred ulps of the largest term, over-estimated by
// ~50x), which is subtracted from k with the 0.01 D margin.  The caller then keeps c without
// walking; any other outcome walks.  (MOPS_PAIR_TEST, defined with the other build switches.)
#if defined(MOPS_PROF)
// Event counters for perf experiments (tools/build_variant.sh -DMOPS_PROF), read back with
// mops_debug_prof: [0] lane-steps, [1] lane walks, [2] lane cell loads, [3] wave-steps,
// [6] cooperative wave-steps (pathline Euler tile), [7] their groups,
// [4] wave-steps with a walk, [5] wave-steps with a cell load.  Never set in a product build.
__device__ unsigned long long g_prof[16];
#endif

template <int MAXV, bool PAIR>
__device__ __forceinline__ int walk(Cell<MAXV>& c, int cell, double x, double y, double z,
                                    const int* __restrict__ cellrec, const double4* __restrict__ cxyz, int C) {
    MOPS_CNT(4, 1);
    constexpr int REC = ((1 + 2 * MAXV) + 3) / 4 * 4;
    constexpr int Q0 = (1 + MAXV) / 4, Q1 = (2 * MAXV) / 4;  // int4 words holding cellsOnCell
    int buf[(Q1 - Q0 + 1) * 4];
    const int4* r4 = reinterpret_cast<const int4*>(cellrec + (int64_t)cell * REC);
#pragma unroll
    for (int q = Q0; q <= Q1; ++q) {
        const int4 v = r4[q];
        buf[4 * (q - Q0)] = v.x; buf[4 * (q - Q0) + 1] = v.y; buf[4 * (q - Q0) + 2] = v.z; buf[4 * (q - Q0) + 3] = v.w;
    }
    int id[MAXV];
    bool ok[MAXV];
    double s[MAXV];
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
        id[k] = buf[1 + MAXV + k - 4 * Q0];
        ok[k] = (k < c.nv) && id[k] >= 0 && id[k] < C;
        // unconditional (clamped) loads, so all centres are in flight at once
        const double4 q = cxyz[ok[k] ? id[k] : cell];
        const double dx = q.x - x, dy = q.y - y, dz = q.z - z;
        s[k] = dx * dx + dy * dy + dz * dz;  // len3(q - p) before its sqrt
    }
    const double4 qc = cxyz[cell];  // c itself, listed last
    const double ex = qc.x - x, ey = qc.y - y, ez = qc.z - z;
    const double sc = ex * ex + ey * ey + ez * ez;
    const double inf = __builtin_huge_val();
    double bs = inf;
#pragma unroll
    for (int k = 0; k < MAXV; ++k)
        if (ok[k] && s[k] < bs) bs = s[k];
    if (sc < bs) bs = sc;
    if (!(bs < inf)) return cell;  // no finite distance: nothing beats DBL_MAX
    // s > thr  =>  sqrt(s) > sqrt(bs) after rounding (relative gap >> 1 ulp);
    // below 2^-900 the product rounds coarsely, so every s there is compared exactly
    const double thr = (bs < 0x1p-900) ? 0x1p-900 : bs * (1.0 + 0x1p-40);
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
        if (ok[k] && s[k] <= thr) {
            if (s[k] == bs || sqrt(s[k]) == sqrt(bs)) return id[k];
        }
    }
    // c attains the minimum and no neighbour ties it (so every finite s_k > s_c)
    double s2 = inf;
    int id1 = -1;  // the nearest neighbour (first of equals)
#pragma unroll
    for (int k = 0; k < MAXV; ++k)
        if (ok[k] && s[k] < s2) { s2 = s[k]; id1 = id[k]; }
    double rb2 = -1.0;
    if (!(s2 < inf)) {
        c.rs2 = inf;  // no neighbour with a finite distance: the walk can only keep c
    } else {
        const double dc = sqrt(sc), d1 = sqrt(s2);
        const double ra = (d1 - dc - 0.01) * 0.5;
        c.rs2 = (ra > 0.0) ? ra * ra * (1.0 - 1e-9) : -1.0;
        if constexpr (PAIR) {
            double s3 = inf;  // the second-nearest distinct neighbour
#pragma unroll
            for (int k = 0; k < MAXV; ++k)
                if (ok[k] && id[k] != id1 && s[k] < s3) s3 = s[k];
            const double rb = (s3 < inf) ? (sqrt(s3) - dc - 0.01) * 0.5 : -1.0;
            if (ra > 0.0 && rb > ra) {
                const double4 q1 = cxyz[id1];
                const double c2 = qc.x * qc.x + qc.y * qc.y + qc.z * qc.z;
                const double c12 = q1.x * q1.x + q1.y * q1.y + q1.z * q1.z;
                const double p2 = x * x + y * y + z * z;
                const double D = 2.0 * rb + dc + d1;
                const double err = 1e-13 * (c2 + c12 + p2 + rb * rb);
                c.pr2[0 * kTrajBlock] = 2.0 * (qc.x - q1.x);
                c.pr2[1 * kTrajBlock] = 2.0 * (qc.y - q1.y);
                c.pr2[2 * kTrajBlock] = 2.0 * (qc.z - q1.z);
                c.pr2[3 * kTrajBlock] = (c12 - c2) - 0.01 * D - err;
                rb2 = rb * rb * (1.0 - 1e-9);
            }
        }
    }
    if constexpr (PAIR) {
        if (MOPS_LDS_COMPACT) *c.rb2 = __double2float_rz(rb2);  // <= rb2: a conservative ball
        else c.pr2[4 * kTrajBlock] = rb2;
    }
    c.cx = x; c.cy = y; c.cz = z;
    return cell;
}

// Exact "c stays" test from the neighbour table (MOPS_NBR_TEST).  With e = p - c,
// d_k = q_k - c and f_k = |d_k|^2 - 2 d_k.e = |p - q_k|^2 - |p - c|^2 (exactly, in real arithmetic), the
// walk keeps c iff every considered neighbour's computed distance stays strictly above c's -- which holds
// when f_k > 0 by more than the rounding of the reference's doubles.  Here f_k is evaluated in float from
// the float offsets: g_k = fl(h_k - 2 fl(d_k.e)), h_k = fl(|d_k|^2), |g_k - f_k| < 2^-20 (h_k + |e|^2)
// (float storage and arithmetic, 12.5 ulp-units at most), so g_k > M_k = 2^-17 (h_k + |e|^2) proves
// f_k > 0.87 M_k, far above the doubles' rounding (2^-50 of the same scale).  Then every p' within
// r = min_k (g_k - M_k) / (2 |d_k|) of p keeps the same margin (f_k moves by <= 2 |d_k| |p' - p|), so the
// test also re-centres the stay ball on p with that radius.  Any other outcome (a bisector within the
// margin, a crossing, a non-finite p) returns false and the caller walks as before.
template <int MAXV, bool PT>
__device__ __forceinline__ bool nbr_stay(Cell<MAXV>& c, int cell, double x, double y, double z,
                                         const uint4* __restrict__ nbr) {
    const uint4* t = nbr + (int64_t)cell * kNbrQ;
    uint32_t w[4 * kNbrQ];
#pragma unroll
    for (int q = 0; q < kNbrQ; ++q) {
        const uint4 v = t[q];
        w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w;
    }
    const double cx = __hiloint2double((int)w[1], (int)w[0]);
    const double cy = __hiloint2double((int)w[3], (int)w[2]);
    const double cz = __hiloint2double((int)w[5], (int)w[4]);
    const float fx = (float)(x - cx), fy = (float)(y - cy), fz = (float)(z - cz);
    const float e2 = fx * fx + fy * fy + fz * fz;
    const uint32_t mask = w[27];
    bool ok = true;
    float r = __builtin_huge_valf();
    float r2 = __builtin_huge_valf(), n1x = 0.0f, n1y = 0.0f, n1z = 0.0f, h1 = 0.0f;  // MOPS_NBR_PAIR
#pragma unroll
    for (int k = 0; k < 7; ++k) {
        if ((mask >> k) & 1u) {
            const float dx = __uint_as_float(w[6 + 3 * k]), dy = __uint_as_float(w[7 + 3 * k]),
                        dz = __uint_as_float(w[8 + 3 * k]);
            const float h = dx * dx + dy * dy + dz * dz;
            const float g = h - 2.0f * (dx * fx + dy * fy + dz * fz);
            const float M = 0x1p-17f * (h + e2);
            ok = ok & (g > M);  // (false for NaN / inf operands)
            const float rk = (g - M) * (0.5f * __builtin_amdgcn_rsqf(h));
            if constexpr (PT && MOPS_NBR_PAIR) {  // the nearest bisector and the second-nearest distance
                const bool nearer = rk < r;
                r2 = nearer ? r : fminf(r2, rk);
                n1x = nearer ? dx : n1x; n1y = nearer ? dy : n1y; n1z = nearer ? dz : n1z; h1 = nearer ? h : h1;
            }
            r = fminf(r, rk);
        }
    }
    if (!ok) return false;
    const double rr = (double)(r * (1.0f - 0x1p-16f));  // (rsq, the products: < 2^-20 relative)
    c.cx = x; c.cy = y; c.cz = z;
    c.rs2 = rr * rr * (1.0 - 1e-9);  // (inf when no neighbour is considered: the walk can only keep c)
    if constexpr (PT) {
        // The pair test's ball is centred on the anchor, which just moved.  MOPS_NBR_PAIR: re-arm it from the
        // table -- inside the ball of the second-nearest bisector's radius r2 only the nearest one, k1, can be
        // crossed, and f_k1(p') = h1 - 2 d1.(p' - c) = n.p' + k with n = -2 d1, k = h1 + 2 d1.c (DESIGN.md
        // section 4.11; the float offsets' error over that ball is below M' / 32)
        float rb2 = -1.0f;
        if constexpr (MOPS_NBR_PAIR) {
            if (r2 > r) {
                const double rr2 = fmin((double)(r2 * (1.0f - 0x1p-16f)), sqrt((double)h1));
                const double Mp = 0x1p-16 * ((double)h1 + 2.0 * (double)e2 * 1.01 + 2.0 * rr2 * rr2);
                const double dx = n1x, dy = n1y, dz = n1z;
                c.pr2[0 * kTrajBlock] = -2.0 * dx;
                c.pr2[1 * kTrajBlock] = -2.0 * dy;
                c.pr2[2 * kTrajBlock] = -2.0 * dz;
                c.pr2[3 * kTrajBlock] = ((double)h1 + 2.0 * (dx * cx + dy * cy + dz * cz)) - Mp;
                rb2 = __double2float_rz(rr2 * rr2 * (1.0 - 1e-9));
            }
        }
        if (MOPS_LDS_COMPACT) *c.rb2 = rb2;
        else c.pr2[4 * kTrajBlock] = rb2;
    }
    return true;
}

template <int MAXV, int NV>
__device__ __forceinline__ bool weights_finite(const Cell<MAXV>& c, const double* w) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < MAXV; ++i)
        if (i < nverts<NV>(c)) ok = ok & isfinite(w[i]);
    return ok;
}

// May the hinted fast bracket (layer_eval / bracket_mono) run for this cell,
// field and particle, and over which levels?  `m` is the field's fast-path
// word for the cell (mono_kernel): every vertex column is either identically
// 0 (a boundary vertex, quirk Q10) or strictly decreasing by >= 1e-6 m per
// level over levels 0..km ("decreasing" vertices, at least one).  Returns km,
// or -1 for "general bracket only".
//
// Why km is exact: with finite weights w_v >= 0 (triangle areas are sqrt's),
// a zero column adds w_v * 0 = +0 to each level sum, i.e. nothing, so the
// computed z_k is the rounded sum over the decreasing vertices only.  Its
// rounding error is below 21 * 2^-53 * sum_dec(w_v |z_v,k|) <= 2.4e-15 * W *
// 1e6 m (|z| <= 1e6 m, <= 20 terms, W = sum of the decreasing vertices'
// weights), while the exact drop z_{k-1} - z_k is >= W * 1e-6 m.  Both scale
// with W, so for every W > 0 the computed column strictly decreases over
// 0..km (drop - 2 * error >= W * (1e-6 - 4.8e-9)); W >= 1e-200 keeps every
// term clear of subnormal rounding.  The reference's fix-up therefore never
// fires there and its bracket predicates are monotone in the level.
template <int MAXV, int NV>
__device__ __forceinline__ int fast_ok(const Cell<MAXV>& c, uint32_t m, bool wfin, const double* w) {
    if (!(m & 0x80000000u) || !wfin) return -1;
    const int km = (int)((m >> 20) & 0x7fu);
    const uint32_t zmask = m & 0x000fffffu;
    if (zmask == 0u) return km;
    double W = 0.0;
#pragma unroll
    for (int i = 0; i < MAXV; ++i)
        if (i < nverts<NV>(c) && !((zmask >> i) & 1u)) W += w[i];
    return (W >= 1e-200) ? km : -1;
}

struct Field {
    const double* __restrict__ zt;   // cellVertexZTop [V][L]
    const double* __restrict__ pr;   // level-pair records [V][L-1][kPairRec] (see mops_field)
};

// Weighted sums of one level-pair record per vertex: everything an
// evaluation needs when the particle's layer is k.  Each sum keeps the
// reference's vertex order, so every value equals its reference counterpart
// (col(), TBBKernel::CalcVelocity, CalcAttribute) bit for bit.
struct Pair {
    double zm, zk;       // z_{k-1}, z_k
    double wm, wk;       // vertical velocity at interfaces k-1, k
    double um0, um1, um2, uk0, uk1, uk2;  // horizontal velocity at levels k-1, k
};

// Weighted sums of the level-pair records of one layer over the stencil.
// Vertices are taken GR at a time under one `v < nv` branch, so GR records are
// in flight per memory round trip (PairGroup: 2 for RK4, whose four
// evaluations per step leave latency exposed; 1 for Euler, where the extra
// VGPRs cost a wave per SIMD -- measured).  A slot v >= nv inside a group reads the all-zero
// record at index V*(L-1) with weight 0 and adds +0.0: a sum that starts at
// +0.0 and only adds products is never -0.0 (x + -x = +0 under
// round-to-nearest) and S + +0.0 == S otherwise (NaN, inf included), so
// every sum keeps the bits of the reference's nv-term loop.
#ifndef MOPS_PAIR_BARRIER
#define MOPS_PAIR_BARRIER 1
#endif
#ifndef MOPS_SCHED_BAR_PR
#define MOPS_SCHED_BAR_PR 1  // the tiled RK4 pathline evaluation keeps the per-slot / per-group scheduling barriers
#endif
#ifndef MOPS_SCHED_BAR_PE
#define MOPS_SCHED_BAR_PE 1  // ... and the tiled Euler one
#endif
template <int MAXV, int GR, int NV, bool COOP = false, bool BAR = true>
__device__ __forceinline__ void pair_sums(const Cell<MAXV>& c, const double* w, const double* __restrict__ pr, int L,
                                          int k, Pair& S, const double2* trec = nullptr) {
    MOPS_MARK(300 + NV);
    S.zm = S.zk = S.wm = S.wk = 0.0;
    S.um0 = S.um1 = S.um2 = S.uk0 = S.uk1 = S.uk2 = 0.0;
    // 32-bit piece indices (mops_mesh_create: pr_pieces < 2^32)
    const uint32_t zrec = pr_zero((uint32_t)c.V, (uint32_t)L), qs = pr_qstride((uint32_t)c.V);
    // tile reads (LDS latency) need fewer records in flight than gathers
    constexpr int GR_ = COOP ? MOPS_GR_COOP : GR;
#pragma unroll
    for (int v0 = 0; v0 < MAXV; v0 += GR_) {
        if (v0 < nverts<NV>(c)) {
            double2 a[GR_][kPairRec / 2];
#pragma unroll
            for (int j = 0; j < GR_; ++j) {
                const int v = v0 + j;
                if (v >= MAXV) break;
#if defined(MOPS_ABL_PAIR1)
            const uint32_t ri = pr_base((uint32_t)(k - 1), (uint32_t)c.vid[0], (uint32_t)c.V);
#else
            const uint32_t ri = (v < nverts<NV>(c)) ? pr_base((uint32_t)(k - 1), (uint32_t)c.vid[v], (uint32_t)c.V) : zrec;
#endif
                if constexpr (COOP) {  // the wave's LDS tile: this vertex's record at the group's layer (zeros past nv)
#pragma unroll
                    for (int q = 0; q < kPairRec / 2; ++q) a[j][q] = trec[(kPairRec / 2) * v + q];
                } else {
                    // (a 64-bit base, then the pieces at q * qs: with record-major records (qs = 1) the five loads
                    // share one address and take immediate offsets)
                    const double2* r = reinterpret_cast<const double2*>(pr) + ri;
#pragma unroll
                    for (int q = 0; q < kPairRec / 2; ++q) a[j][q] = r[(size_t)q * qs];
                }
            }
#pragma unroll
            for (int j = 0; j < GR_; ++j) {
                const int v = v0 + j;
                if (v >= MAXV) break;
                const double wv = w[v];
                S.zm += wv * a[j][0].x; S.zk += wv * a[j][0].y;
                S.wm += wv * a[j][1].x; S.wk += wv * a[j][1].y;
                S.um0 += wv * a[j][2].x; S.um1 += wv * a[j][2].y; S.um2 += wv * a[j][3].x;
                S.uk0 += wv * a[j][3].y; S.uk1 += wv * a[j][4].x; S.uk2 += wv * a[j][4].y;
            }
            // NV > 0 has no per-group branch: keep the groups apart, or the
            // scheduler puts every record in flight at once and spills
            if constexpr ((NV > 0 || COOP) && MOPS_PAIR_BARRIER && BAR) __builtin_amdgcn_sched_barrier(0);
        }
    }
    MOPS_MARK(310 + NV);
}

// Layer + values for one field.  Fast path (fast_ok gave the decreasing
// prefix km >= 1 and the hint h is in 1..km): ONE record per vertex decides
// whether the layer is h -- Q(h), !Q(h-1), !P(h+1) (notation of
// bracket_scan), i.e. a = b = h, which both the binary search (streamline)
// and the linear scan (pathline) resolve to h; the record's z_{h-1}, z_h are
// the fixed-up z'_{h-1}, z'_h because h <= km -- plus the reference's "above
// the surface" test d > z_0 + eps first.  That test needs no z_0 in the
// record: for h == 1, z_0 = z_{h-1}; for h >= 2 the accepted case has d <
// z_{h-1} - eps < z_0 - eps (strictly decreasing prefix), so d > z_0 + eps is
// false there.  A particle below the bottom of a fully decreasing column
// (km = L-1) is accepted at h = L-1 the same way (the reference's "below the
// bottom" branch).  Otherwise bracket_mono walks from the hint inside the prefix,
// and bracket_scan (the whole fixed-up column) runs when the walk would leave
// it; the record of the final layer is then read.
template <int MAXV, bool PATH, int GR, int NV, bool COOP = false, bool TCHK = false>
__device__ __forceinline__ int layer_eval(const Cell<MAXV>& c, const double* w, int km, const Field& f, int L,
                                          double d, int& hint, Pair& S, const double2* trec = nullptr,
                                          int th = 0) {
    const double eps = 1e-8;
    const int h = hint;
    if (h >= 1 && h <= km) {  // km = -1: general bracket only (fast_ok)
        // (a cooperative wave's tile holds every vertex's record at the layer the lane's hint had when
        // the tile was filled, th: always this one in Euler; an RK4 stage after another stage moved
        // the hint (TCHK) gathers its records itself -- the next step regroups the wave)
        if constexpr (COOP && TCHK) {
            if (h == th) pair_sums<MAXV, GR, NV, true, MOPS_SCHED_BAR_PR>(c, w, f.pr, L, h, S, trec);
            else pair_sums<MAXV, GR, NV>(c, w, f.pr, L, h, S);
        } else {
            pair_sums<MAXV, GR, NV, COOP, (!COOP || MOPS_SCHED_BAR_PE)>(c, w, f.pr, L, h, S, trec);
        }
        bool ok;
        if (h == 1 && d > S.zm + eps) {  // above the surface (z_0 = z_{h-1} here)
            ok = true;
        } else if (h == L - 1 && km == L - 1 && d < S.zk - eps) {
            // below the bottom: !Q(L-1) with the whole column decreasing -- the
            // reference's "below the bottom" branch, layer L-1 with z'_{L-1} = z_{L-1}
            // and z'_{L-2} = z_{L-2} (bracket_mono's not-found case)
            ok = true;
        } else {
            const bool Qh = d >= S.zk - eps;
            const bool Qm = (h > 1) && (d >= S.zm - eps);
            const bool Pn = (h < L - 1) && (d <= S.zk + eps);
            ok = Qh && !Qm && !Pn;
        }
        if (ok) return h;
    }
    MOPS_CNT(6, 1);
    double zdn, zup;
    int layer = -2;
    if (km >= 1) layer = bracket_mono<MAXV, PATH>(c, w, f.zt, L, km, d, hint, zdn, zup);
    if (layer == -2) {
        layer = bracket_scan<MAXV, PATH>(c, w, f.zt, L, d, zdn, zup);
        hint = layer;
    }
    if (layer < 0) return -1;
    pair_sums<MAXV, GR, NV>(c, w, f.pr, L, layer, S);
    S.zk = zdn;  // the bracket's (possibly fixed-up) column values
    S.zm = zup;
    return layer;
}

// streamline calc_velocity_at (MPASOVisualizerKernels.cpp:740-872)
template <int MAXV, int GR, int NV>
__device__ __forceinline__ bool eval_stream(const Cell<MAXV>& c, int L, int V, const Field& f, double px, double py,
                                            double pz, double d, int& hint, double& hx, double& hy, double& hz,
                                            double& wv) {
    double w[MAXV];
    MOPS_MARK(400 + NV);
    if (!weights<MAXV, NV>(c, L, V, px, py, pz, w)) return false;
    Pair S;
    MOPS_MARK(410 + NV);
    const int layer = layer_eval<MAXV, false, GR, MOPS_HEX_PAIRS ? NV : 0>(c, w, fast_ok<MAXV, NV>(c, c.mono0, weights_finite<MAXV, NV>(c, w), w), f,
                                                  L, d, hint, S);
    MOPS_MARK(420 + NV);
    if (layer < 0) return false;
    const double zdn = S.zk, zup = S.zm;
    double x = d;
    x = dmax(zdn, dmin(x, zup));
    const double den = zup - zdn;
    if (fabs(den) < 1e-12) return false;
    const double t = (x - zdn) / den;
    // vel_dn at `layer`, vel_up at `layer - 1`; w at interfaces layer, layer-1
    if (sq3(S.uk0, S.uk1, S.uk2) < kNormTiny2 || sq3(S.um0, S.um1, S.um2) < kNormTiny2) return false;
    hx = S.um0 * t + S.uk0 * (1.0 - t);
    hy = S.um1 * t + S.uk1 * (1.0 - t);
    hz = S.um2 * t + S.uk2 * (1.0 - t);
    if (sq3(hx, hy, hz) < kNormTiny2) return false;
    wv = t * S.wm + (1.0 - t) * S.wk;
    MOPS_MARK(430 + NV);
    return true;
}

// pathline calc_velocity_at (MPASOVisualizerKernels.cpp:1124-1327).  The
// attribute channel is not evaluated: FinalizeTrajectoryLinesWithAttrs never
// reads it (TrajectoryCommon.h:176-185, quirk Q9), so it is unobservable.
template <int MAXV, int GR, int NV, bool COOP = false, bool TCHK = false>
__device__ __forceinline__ bool eval_path(const Cell<MAXV>& c, int L, int V, const Field& ff, const Field& fb,
                                          double px, double py, double pz, double d, double alpha, int& hint0,
                                          int& hint1, double& hx, double& hy, double& hz, double& wv,
                                          const double2* tile = nullptr, int th0 = 0, int th1 = 0) {
    double w[MAXV];
    constexpr bool kBar = !COOP || (TCHK ? MOPS_SCHED_BAR_PR : MOPS_SCHED_BAR_PE);
    if (!weights<MAXV, NV, COOP, kBar>(c, L, V, px, py, pz, w, reinterpret_cast<const double4*>(tile))) return false;
    const bool wfin = weights_finite<MAXV, NV>(c, w);
    Pair F, B;
    const int lf = layer_eval<MAXV, true, GR, MOPS_HEX_PAIRS_P ? NV : 0, COOP, TCHK>(
        c, w, fast_ok<MAXV, NV>(c, c.mono0, wfin, w), ff, L, d, hint0, F, tile + kTileOffRec, th0);
    const int lb = layer_eval<MAXV, true, GR, MOPS_HEX_PAIRS_P ? NV : 0, COOP, TCHK>(
        c, w, fast_ok<MAXV, NV>(c, c.mono1, wfin, w), fb, L, d, hint1, B, tile + kTileOffRec + kTileRec, th1);
    if (lf < 0 || lb < 0) return false;
    const double xf = dmax(F.zk, dmin(d, F.zm));
    const double denf = F.zm - F.zk;
    if (fabs(denf) < 1e-12) return false;
    const double tf = (xf - F.zk) / denf;
    const double xb = dmax(B.zk, dmin(d, B.zm));
    const double denb = B.zm - B.zk;
    if (fabs(denb) < 1e-12) return false;
    const double tb = (xb - B.zk) / denb;
    const double fx = F.um0 * tf + F.uk0 * (1.0 - tf), fy = F.um1 * tf + F.uk1 * (1.0 - tf),
                 fz = F.um2 * tf + F.uk2 * (1.0 - tf);
    const double gx = B.um0 * tb + B.uk0 * (1.0 - tb), gy = B.um1 * tb + B.uk1 * (1.0 - tb),
                 gz = B.um2 * tb + B.uk2 * (1.0 - tb);
    hx = gx * alpha + fx * (1.0 - alpha);
    hy = gy * alpha + fy * (1.0 - alpha);
    hz = gz * alpha + fz * (1.0 - alpha);
    const double wf = tf * F.wm + (1.0 - tf) * F.wk;
    const double wb = tb * B.wm + (1.0 - tb) * B.wk;
    wv = alpha * wb + (1.0 - alpha) * wf;
    return true;
}

// One velocity evaluation.  A wave whose lanes all sit in hexagons (the bulk
// of an MPAS mesh) runs the NV = 6 instantiation; any other wave the general
// one.  Both compute the same operations in the same order.
#ifndef MOPS_HEX_PR_COOP
#define MOPS_HEX_PR_COOP 1  // the pathline RK4 kernel's tile evaluation has an NV = 6 instantiation
#endif
#ifndef MOPS_HEX_PR_PLAIN
#define MOPS_HEX_PR_PLAIN 1  // ... and its per-lane evaluation
#endif
template <int MAXV, bool PATH, int GR, bool TCHK = false, bool HEXTILE = false>
__device__ __forceinline__ bool eval_at(bool hex, const Cell<MAXV>& c, int L, int V, const Field& f0,
                                        const Field& f1, double px, double py, double pz, double d, double alpha,
                                        int& hint0, int& hint1, double& hx, double& hy, double& hz, double& wv,
                                        bool coop = false, const double2* tile = nullptr, int th0 = 0, int th1 = 0) {
    // (TCHK: the RK4 pathline kernels, four inlined evaluations per step -- code size; see MOPS_HEX_PR_*)
    // (HEXTILE: the hand-off RK4 kernel, whose waves are all cooperative and hexagonal -- the only instantiation)
    if constexpr (HEXTILE) {
        static_assert(MAXV == 7 && PATH, "the hexagon tile evaluation is the MAXV 7 pathline one");
        return eval_path<MAXV, GR, 6, true, TCHK>(c, L, V, f0, f1, px, py, pz, d, alpha, hint0, hint1, hx, hy, hz, wv,
                                                  tile, th0, th1);
    }
    if constexpr (MAXV == 7 && PATH) {
        if (coop) {  // wave-uniform: the tile instantiations
            if ((MOPS_HEX_PR_COOP || !TCHK) && hex) return eval_path<MAXV, GR, 6, true, TCHK>(c, L, V, f0, f1, px, py, pz, d, alpha, hint0, hint1, hx,
                                                               hy, hz, wv, tile, th0, th1);
            return eval_path<MAXV, GR, 0, true, TCHK>(c, L, V, f0, f1, px, py, pz, d, alpha, hint0, hint1, hx, hy, hz,
                                                      wv, tile, th0, th1);
        }
    }
    if constexpr (MAXV == 7) {
        if ((MOPS_HEX_PR_PLAIN || !(PATH && TCHK)) && hex)
            return PATH ? eval_path<MAXV, GR, 6>(c, L, V, f0, f1, px, py, pz, d, alpha, hint0, hint1, hx, hy, hz, wv)
                        : eval_stream<MAXV, GR, 6>(c, L, V, f0, px, py, pz, d, hint0, hx, hy, hz, wv);
    }
    return PATH ? eval_path<MAXV, GR, 0>(c, L, V, f0, f1, px, py, pz, d, alpha, hint0, hint1, hx, hy, hz, wv)
                : eval_stream<MAXV, GR, 0>(c, L, V, f0, px, py, pz, d, hint0, hx, hy, hz, wv);
}

}  // namespace dev

// ===========================================================================
// trajectory kernel
// ===========================================================================
struct TrajArgs {
    const int* __restrict__ cellrec;
    const double4* __restrict__ cxyz;
    const double4* __restrict__ vxyz;
    int C, V, L;
    dev::Field f0, f1;
    const uint32_t* __restrict__ mono0;
    const uint32_t* __restrict__ mono1;
    const int* __restrict__ order;  // slot -> particle (NULL = identity)
    const int* __restrict__ n_live;  // device count of leading live slots (compaction), NULL = all n
    const double4* __restrict__ cpoly;  // per-cell rotated polygon + Wachspress B_i (mops_mesh::d_cpoly)
    const double* __restrict__ cnrm;    // per-cell edge normals (mops_mesh::d_cnrm; NULL past maxEdges 7)
    const double* __restrict__ cedge;   // per-cell edge vectors (mops_mesh::d_cedge; MOPS_TILE_E1 only)
    const uint4* __restrict__ nbr;      // per-cell neighbour table (mops_mesh::d_nbr; NULL past maxEdges 7)
    const double2* __restrict__ cpolyr;  // mops_mesh::d_cpolyr (NULL past maxEdges 7)
    const uint32_t* __restrict__ crank;  // mops_mesh::d_cell_rank
    const int* __restrict__ coop_sel;   // per-launch device flag: 1 = the cooperative instantiation runs, 0 = the
                                        // plain one (the other exits at once); NULL = no selection
    int handoff;          // pathline RK4: the hand-off kernel runs first, the cooperative one resumes its waves
    double* px; double* py; double* pz;
    float* depth;
    int* cell;
    int* death;
    int64_t n;
    int64_t step_begin, step_end, n_steps;
    int delta_t;          // signed (dt_sign * deltaT)
    double dalpha;        // pathline RK4: dt / simulationDuration
    int64_t rec_period;   // record at step j iff (j+1) % rec_period == 0 (0 = never)
    int64_t K;
    double* rec;
    int64_t rec_stride;
};

// One piece of a cooperative wave's tile (traj_kernel's regroup): piece pc of group gg -- the polygon, the
// edge normals, the front field's records, the back field's -- from the group headers hdi into s_tile[i]
template <int MAXV>
__device__ __forceinline__ void tile_piece(int i, const uint32_t* hdi, const double2* cpoly2, const double2* cnrm2,
                                           const double2* cedge2, const double2* pr0, const double2* pr1, uint32_t V,
                                           double2* s_tile) {
    const int gg = i / kTilePieces, pc = i - gg * kTilePieces;
    const uint32_t cl = hdi[gg * kTileHdr];
    const bool isp = pc < kTileOffNrm, isn = pc < kTileOffRec;
    const bool f1 = pc >= kTileOffRec + kTileRec;
    const int pp = isn ? 0 : pc - (f1 ? kTileOffRec + kTileRec : kTileOffRec);
    const int v = pp / (kPairRec / 2), q = pp - (kPairRec / 2) * v;
    const uint32_t ri = hdi[gg * kTileHdr + 4 + (f1 ? 8 : 0) + v];
    const bool ise = MOPS_TILE_E1 && pc >= kTileOffE1;  // (with isn: an edge-vector piece)
    const double2* base = isp ? cpoly2 : (isn ? (ise ? cedge2 : cnrm2) : (f1 ? pr1 : pr0));
    const uint64_t idx = isp ? ((uint64_t)cl * MAXV + (uint32_t)(pc >> 1)) * 2 + (uint32_t)(pc & 1)
                             : (isn ? (uint64_t)cl * kCellNrmPieces +
                                          (uint32_t)(pc - (ise ? kTileOffE1 : kTileOffNrm))
                                    : (uint64_t)(ri + (uint32_t)q * pr_qstride(V)));
    s_tile[i] = base[idx];
}

// Minimum waves per SIMD requested per instantiation (register budget vs
// latency hiding; swept on MI355X with tools/occupancy_sweep.sh).
#ifndef MOPS_W_SE
#define MOPS_W_SE 3  // streamline Euler
#endif
#ifndef MOPS_W_SR
#define MOPS_W_SR 2  // streamline RK4 (at 1 the shared-reciprocal normalisation took it to 260 VGPRs = 1 wave)
#endif
#ifndef MOPS_W_PE
#define MOPS_W_PE 3  // pathline Euler (at 1 the compiler takes 172 VGPRs = 2 waves: -9.5% at config 2's mesh)
#endif
#ifndef MOPS_W_PR
#define MOPS_W_PR 2  // pathline RK4
#endif
#ifndef MOPS_RK4_LOOP
#define MOPS_RK4_LOOP 0  // 1: RK4 stages as a loop around one inlined evaluation (4x less code, but 220-240 spilled
                         // VGPRs: pathline RK4 5.34e9 vs 6.97e9, streamline RK4 3.5e9 vs 6.9e9 p-steps/s, measured)
#endif
#ifndef MOPS_RK4_ACC
#define MOPS_RK4_ACC 1  // RK4 stage velocities accumulated as they come (see traj_kernel)
#endif
#ifndef MOPS_RK4_FENCE
#define MOPS_RK4_FENCE 0  // a compiler memory barrier between RK4 stages: each stage re-reads the cell's polygon,
                          // normals and tile records instead of keeping stage 1's loads live across the step
#endif
#if MOPS_RK4_FENCE
#define MOPS_STAGE_FENCE() asm volatile("" ::: "memory")
#else
#define MOPS_STAGE_FENCE() do { } while (0)
#endif
#ifndef MOPS_GR_E
#define MOPS_GR_E 1  // level-pair records in flight per round trip, Euler
#endif
#ifndef MOPS_GR_R
#define MOPS_GR_R 2  // RK4
#endif
#ifndef MOPS_GR_PE
#define MOPS_GR_PE 2  // pathline Euler (with the NV = 6 pair sums: 44.6 vs 45.7 ms at GR 1, config 2 mesh)
#endif
template <bool PATH, bool EULER>
struct PairGroup {
    static constexpr int value = EULER ? (PATH ? MOPS_GR_PE : MOPS_GR_E) : MOPS_GR_R;
};
// Wide stencils (maxEdges > 7: MAXV 12 / 20) never cache the polygon in
// registers and ask for fewer waves -- their per-vertex arrays alone would
// otherwise spill.
template <int MAXV, bool PATH, bool EULER>
struct RCache {
    static constexpr bool value =
        MAXV <= 7 && (PATH ? (EULER ? MOPS_RC_PE : MOPS_RC_PR) : (EULER ? MOPS_RC_SE : MOPS_RC_SR));
};
// The polygon's IsInMesh edge normals kept in LDS (10.5 KB per 64-lane block),
// computed at each cell change instead of per evaluation: 27.9 vs 29.0 ms (SE)
// at config 2.  In streamline RK4 the extra registers first crossed 256 VGPRs
// (1 wave per SIMD, 135 vs 92 ms); with the RK4 kernels held at 2 waves/SIMD by
// their launch bounds (MOPS_W_SR 2) they fit, and all four modes use them.
#ifndef MOPS_NRM_SE
#define MOPS_NRM_SE 1
#endif
#ifndef MOPS_NRM_PE
#define MOPS_NRM_PE 1
#endif
#ifndef MOPS_NRM_PE_PLAIN
// the plain (not cooperative) pathline Euler kernel, which runs the sparse waves of config 4, computes its
// normals per evaluation instead: since the neighbour-table test the per-cell LDS column no longer pays --
// config 4 2841 -> 2797 ms per 6-pair chain (3 interleaved rounds), config-2 mesh pathline 38.2-38.8 ms
// either way (profiles/r05/ab/plain_kernel_normals.txt)
#define MOPS_NRM_PE_PLAIN 0
#endif
#ifndef MOPS_NRM_SR
#define MOPS_NRM_SR 1  // with MOPS_W_SR 2 capping it at 256 VGPRs: 86.3-87.0 vs 88.6-89.2 ms (config-2 mesh)
#endif
#ifndef MOPS_NRM_PR
#define MOPS_NRM_PR 1  // 125.7 vs 127.2 ms
#endif
template <int MAXV, bool PATH, bool EULER>
struct LdsNormals {
    static constexpr bool value =
        MAXV <= 7 && (EULER ? (PATH ? MOPS_NRM_PE : MOPS_NRM_SE) : (PATH ? MOPS_NRM_PR : MOPS_NRM_SR));
};
#ifndef MOPS_W_PE_PLAIN
#define MOPS_W_PE_PLAIN MOPS_W_PE  // the plain (not cooperative) pathline Euler kernel
#endif
#ifndef MOPS_RK4_HANDOFF
#define MOPS_RK4_HANDOFF 1  // pathline RK4: a hexagon-tile-only kernel at MOPS_W_PR_HAND waves first (see traj_kernel):
                            // config-3 RK4 launch 289 vs 313 ms, 7.42e9 vs 6.87e9 p-steps/s (2 interleaved rounds);
                            // with the tile filled past MOPS_COOP_R pieces per lane there, 287.5 vs 289 ms
#endif
#ifndef MOPS_W_PR_HAND
#define MOPS_W_PR_HAND 3
#endif
template <int MAXV, bool PATH, bool EULER, bool COOP = false, bool HAND = false>
struct TrajWaves {
    static constexpr int base = PATH ? (EULER ? (COOP ? MOPS_W_PE : MOPS_W_PE_PLAIN) : (HAND ? MOPS_W_PR_HAND : MOPS_W_PR))
                                     : (EULER ? MOPS_W_SE : MOPS_W_SR);
    static constexpr int value = MAXV <= 7 ? base : (EULER ? 2 : 1);
};

// HAND (pathline RK4, MOPS_RK4_HANDOFF): the hand-off kernel.  It holds only the hexagon tile evaluation --
// the cooperative kernel's other two (the general-polygon tile, the per-lane one) are what keep that kernel at
// 2 waves/SIMD -- and runs a wave while every step finds it cooperative and hexagonal.  At the first step that
// does not, the wave stops before the step's walk takes effect and hands over: its state is the step's start
// (position, depth, the cell the walk starts from) and death[pid] = -2 - step marks where to resume.  The
// cooperative kernel, launched after it (TrajArgs::handoff), runs only such waves, from that step on: the same
// as a launch boundary at that step for them (the walk's shortcuts, the hints and the tile are exact or speed
// only), so records and states are the same bits as one kernel's.
template <int MAXV, bool PATH, bool EULER, bool COOP = false, bool HAND = false>
__global__ void __launch_bounds__(kTrajBlock, (TrajWaves<MAXV, PATH, EULER, COOP, HAND>::value)) traj_kernel(TrajArgs a) {
    static_assert(!HAND || (MAXV == 7 && PATH && !EULER && COOP), "the hand-off kernel is the pathline RK4 tile one");
    if (a.coop_sel && ((*a.coop_sel != 0) != COOP)) return;  // the other instantiation runs this launch
    // XCD-aware mapping: blocks b, b+8, ... share an XCD (L2); give each XCD a
    // contiguous range of the locality-ordered particles (bijective remap)
    // After a compaction only the first *n_live slots hold live particles: the remap then spreads
    // just those blocks over the 8 XCDs (blocks beyond them exit at once), instead of handing the
    // dead tail's blocks -- a contiguous range -- to whole XCDs that would sit idle
    unsigned nblk = gridDim.x;
    int64_t n = a.n;
    if (a.n_live) {
        const int64_t nl = *a.n_live;
        n = nl < n ? nl : n;
        nblk = (unsigned)((n + blockDim.x - 1) / blockDim.x);
    }
    const unsigned b = blockIdx.x;
    if (b >= nblk) return;
    const unsigned xcd = b % 8u, q = nblk / 8u, r = nblk % 8u;
    const unsigned blk = (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + b / 8u;
    const int64_t slot = (int64_t)blk * blockDim.x + threadIdx.x;
    if (slot >= n) return;
#if defined(MOPS_WAVE_STAMPS)
    unsigned long long* stamp = dev::stamp_slot();
    if (stamp) {
        stamp[0] = __builtin_amdgcn_s_memrealtime();
        stamp[2] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
        stamp[3] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
        stamp[1] = stamp[0];
    }
    struct StampEnd {
        unsigned long long* p;
        __device__ ~StampEnd() { if (p) p[1] = __builtin_amdgcn_s_memrealtime(); }
    } stamp_end{stamp};
#endif
    const int64_t pid = a.order ? (int64_t)a.order[slot] : slot;
    // the cooperative kernel after the hand-off kernel: only the waves it handed over, each from its step (one
    // per wave: a wave's lanes stop together, and the two kernels map the same slots to a wave); a dead lane's
    // records were cleared by the hand-off kernel, a finished one is done.  (The register allocation of the Euler
    // kernel is sensitive to the form of this prologue and of the epilogue: 128 instead of 70 spilled VGPRs.)
    const bool resumed = COOP && !HAND && !EULER && a.handoff;
    if (resumed && a.death[pid] > -2) return;
    const int64_t sb = resumed ? (int64_t)__builtin_amdgcn_readfirstlane(-2 - a.death[pid]) : a.step_begin;
    // Records need no initialisation: the launches from step 0 on write every record of every
    // particle -- its samples while alive, then (at its death) the zeros the reference's
    // preallocated trajectory holds (dev::clear_records)
    if (a.death[pid] >= 0) {  // the reference's lambda has returned
        if (a.step_begin == 0) dev::clear_records(a.rec, a.rec_stride, pid, 0, a.K);
        return;
    }
    double x = a.px[pid], y = a.py[pid], z = a.pz[pid];
    float dep = a.depth[pid];
    int cell = a.cell[pid];
    int died = -1;
    int hint0 = -1, hint1 = -1;  // previous layer per field (speed only)
    dev::Cell<MAXV> c;
    c.id = -1;
    c.nv = 0;
    c.V = a.V;
    c.cpolyr = a.cpolyr;
    c.crank = a.crank;
    c.C = (uint32_t)a.C;
    // cooperative waves (see kTilePieces): the wave's LDS tile and its group headers; their kernel keeps no
    // per-lane normals (a tiled wave reads its cells' normals from the tile, any other wave computes them)
    // (RK4 too: its four stages are evaluated in the step's start cell, quirk Q1, so a group's polygon and
    // normals hold for the whole step; a stage whose hint left the tile's layer gathers its own records)
    // (MOPS_RC_PE_PLAIN: the plain -- not cooperative -- pathline Euler kernel, which runs the sparse waves of
    // config 4, keeps the polygon in registers: 12 fewer VMEM per evaluation for a TD-bound launch)
    constexpr bool kRC = RCache<MAXV, PATH, EULER>::value || (MOPS_RC_PE_PLAIN && PATH && EULER && !COOP && MAXV <= 7),
                   kNrm = LdsNormals<MAXV, PATH, EULER>::value && (MOPS_NRM_PE_PLAIN || COOP || !PATH || !EULER);
    constexpr bool kCoop = COOP && PATH && MAXV == 7 && !kRC && kNrm && MOPS_CPOLY &&
                           (EULER ? MOPS_COOP_PE : MOPS_COOP_PR);
    // the tile and its headers are per block, and the group/header hand-offs between lanes rely on one
    // wave's LDS operations running in order: one wave per block
    static_assert(!kCoop || kTrajBlock == 64, "the cooperative tile needs one wave per block");
    constexpr bool kNbrT = MOPS_NBR_TEST && MAXV == 7 && (EULER || MOPS_NBR_RK4);  // dev::nbr_stay before a walk
    // per-lane edge normals (Cell::nrm); in the cooperative kernel the same LDS holds either them (a wave in
    // lane-normal mode, c.lds_n) or the wave's tile
    // groups per tile and tile pieces per live lane at most (per kernel: the RK4 one has LDS to spare)
    constexpr int kG = EULER ? MOPS_COOP_G : ((HAND || !MOPS_RK4_HANDOFF) ? MOPS_COOP_G_PR : MOPS_COOP_G_PRR),
                  kR = EULER ? MOPS_COOP_R : MOPS_COOP_R_PR;
    constexpr bool kFillAll = HAND || (!EULER && MOPS_COOP_G_PRR != MOPS_COOP_G_PR);  // (see the tile fill)
    static_assert(kG <= 254, "group index in tkey's low byte (0xff = no tile)");
    constexpr int kNrmD = 3 * kNrmSlots(MAXV) * kTrajBlock, kTileD = 2 * kG * kTilePieces;
    __shared__ __attribute__((aligned(16))) double s_nrm[kNrm ? (kCoop && kTileD > kNrmD ? kTileD : kNrmD) : 1];
    c.nrm = s_nrm + threadIdx.x;
    c.lds_n = kNrm && !kCoop;  // (the cooperative kernel starts in tile mode)
    constexpr bool kPairT = (kNrm || kCoop) && (PATH ? MOPS_PAIR_TEST_P : MOPS_PAIR_TEST);  // (load_cell resets it)
    __shared__ double s_pr2[kPairT ? (MOPS_LDS_COMPACT ? 4 : 5) * kTrajBlock : 1];  // per-lane pair test (Cell::pr2, dev::walk)
    __shared__ float s_rb2[kPairT && MOPS_LDS_COMPACT ? kTrajBlock : 1];
    c.pr2 = s_pr2 + threadIdx.x;
    c.rb2 = s_rb2 + (kPairT && MOPS_LDS_COMPACT ? threadIdx.x : 0);
    double2* s_tile = reinterpret_cast<double2*>(s_nrm);
    __shared__ uint4 s_hdr[kCoop ? kG * (kTileHdr / 4) : 1];
    const int C = a.C;
    // next recording step (the smallest j >= step_begin with (j+1) % rec_period == 0) and its
    // record index, advanced by counting instead of a 64-bit modulo per step
    int64_t rec_next = -1, rec_k = 0;
    bool rec0 = sb > 0;  // record 0's step-0 part (seed position, zero velocity) written
    if (a.rec_period > 0) {
        rec_k = sb / a.rec_period;
        rec_next = (rec_k + 1) * a.rec_period - 1;
    }
    [[maybe_unused]] int cell_in = 0;       // HAND: the cell this step's walk started from
    int tcell = -1, tkey = 0;               // cooperative tile: this lane's (cell, hints) at the last fill + group
    bool have_tile = false, coop_prev = false;  // (wave-uniform)
    for (int64_t step = sb; step < a.step_end; ++step) {
        MOPS_MARK(100);
        if constexpr (HAND) cell_in = cell;  // (the walk restarts from it at a hand-off)
        if (step == 0) {  // first_loop (:892-901)
            if (cell < 0 || cell >= C) { died = 0; break; }
            dev::load_cell<MAXV, kRC, kNrm, kPairT, kCoop>(c, cell, a.cellrec, a.vxyz, a.mono0, a.mono1, a.cxyz, a.cpoly, a.cnrm);
            double* r0 = a.rec;
            r0[0 * a.rec_stride + pid] = x;
            r0[1 * a.rec_stride + pid] = y;
            r0[2 * a.rec_stride + pid] = z;
            r0[3 * a.rec_stride + pid] = 0.0;  // (first_vel below, once step 0 evaluates)
            r0[4 * a.rec_stride + pid] = 0.0;
            r0[5 * a.rec_stride + pid] = 0.0;
            rec0 = true;
        } else {  // one-hop nearest-centre walk (:902-922)
            if (cell < 0 || cell >= C) { died = (int)step; break; }
            if (c.id != cell) dev::load_cell<MAXV, kRC, kNrm, kPairT, kCoop>(c, cell, a.cellrec, a.vxyz, a.mono0, a.mono1, a.cxyz, a.cpoly, a.cnrm);
            // Exact shortcut: inside the stay ball around the anchor every
            // neighbour is strictly farther than c by more than rounding, so
            // the reference's argmin (c listed last, strict <) keeps c (dev::walk).
            const double ex = x - c.cx, ey = y - c.cy, ez = z - c.cz;
#if defined(MOPS_PROF)
            const double e2p = ex * ex + ey * ey + ez * ez;
            bool stay_p = e2p < c.rs2;
            if constexpr (kPairT) {
                if (!stay_p && e2p < (MOPS_LDS_COMPACT ? (double)*c.rb2 : c.pr2[4 * kTrajBlock]))
                    stay_p = c.pr2[0] * x + c.pr2[kTrajBlock] * y + c.pr2[2 * kTrajBlock] * z +
                             c.pr2[3 * kTrajBlock] > 0.0;
            }
            if constexpr (kNbrT) {
                if (!stay_p && dev::nbr_stay<MAXV, kPairT>(c, cell, x, y, z, a.nbr)) {
                    stay_p = true;
                    atomicAdd(&dev::g_prof[13], 1ull);  // lane-steps the neighbour table kept in c
                }
            }
            const bool walking = !stay_p;
            bool loading = false;
            if (walking) {
                cell = dev::walk<MAXV, kPairT>(c, cell, x, y, z, a.cellrec, a.cxyz, C);
                loading = c.id != cell;
                if (c.id != cell) dev::load_cell<MAXV, kRC, kNrm, kPairT, kCoop>(c, cell, a.cellrec, a.vxyz, a.mono0, a.mono1, a.cxyz, a.cpoly, a.cnrm);
            }
            {
                const unsigned long long bw = __ballot(walking), bl = __ballot(loading), ba = __ballot(1);
                if ((int)__lane_id() == __builtin_ffsll((long long)ba) - 1) {
                    atomicAdd(&dev::g_prof[0], (unsigned long long)__popcll(ba));
                    atomicAdd(&dev::g_prof[1], (unsigned long long)__popcll(bw));
                    atomicAdd(&dev::g_prof[2], (unsigned long long)__popcll(bl));
                    atomicAdd(&dev::g_prof[3], 1ull);
                    atomicAdd(&dev::g_prof[4], bw ? 1ull : 0ull);
                    atomicAdd(&dev::g_prof[5], bl ? 1ull : 0ull);
                }
            }
#else
            const double e2 = ex * ex + ey * ey + ez * ez;
            bool stay = e2 < c.rs2;
            if constexpr (kPairT) {
                if (!stay && e2 < (MOPS_LDS_COMPACT ? (double)*c.rb2 : c.pr2[4 * kTrajBlock]))  // second ball: only nb1 competes (dev::walk)
                    stay = c.pr2[0] * x + c.pr2[kTrajBlock] * y + c.pr2[2 * kTrajBlock] * z +
                           c.pr2[3 * kTrajBlock] > 0.0;
            }
            if constexpr (kNbrT) {
                if (!stay) stay = dev::nbr_stay<MAXV, kPairT>(c, cell, x, y, z, a.nbr);  // exact: every bisector clear
            }
#if defined(MOPS_ABL_NOWALK)  // ablation: never walk (wrong results; the walks' cost bound)
            if (false) {
#else
            if (!stay) {
#endif
#if defined(MOPS_ABL_WALK2)  // ablation: every walk runs twice (same result; one walk's cost)
                {
                    double xo = x;
                    asm volatile("" : "+v"(xo));
                    cell = dev::walk<MAXV, kPairT>(c, cell, xo, y, z, a.cellrec, a.cxyz, C);
                }
#endif
                cell = dev::walk<MAXV, kPairT>(c, cell, x, y, z, a.cellrec, a.cxyz, C);
                if (c.id != cell) MOPS_CNT(5, 1);
                if (c.id != cell) dev::load_cell<MAXV, kRC, kNrm, kPairT, kCoop>(c, cell, a.cellrec, a.vxyz, a.mono0, a.mono1, a.cxyz, a.cpoly, a.cnrm);
            }
#endif
        }
        MOPS_MARK(110);
        const double d = -1.0 * (double)dep;
        const double r = dev::len3(x, y, z);
        const bool hex = MOPS_HEX && __all(c.nv == 6);  // wave-uniform (dev::eval_at)
        bool coop = false;  // wave-uniform: this step's polygon and hinted-layer records come from s_tile
        const double2* tile = nullptr;
        if constexpr (kCoop) {
            // The tile persists across steps: within a launch the fields are fixed, so a group's pieces
            // stay valid while no live lane changes its (cell, hint0, hint1) -- cells change ~once per
            // particle-day at config 3.  Any change regroups the wave and refills the whole tile.
            const int hk = ((hint0 + 1) << 16) | ((hint1 + 1) << 8);  // (hints >= -1, < 2^7)
            const bool moved = (cell != tcell) | (hk != (tkey & ~0xff));
            // tile mode: regroup when a lane moved; lane-normal mode (a wave with too many groups): try
            // again every 64 steps
            const bool regroup = c.lds_n ? ((step - sb) & (MOPS_COOP_RETRY - 1)) == 0
                                         : (__ballot(moved) != 0ull || !have_tile);
            if (regroup) {
                // groups of live lanes with equal (cell, hint0, hint1), found leader by leader with
                // scalar readlanes + ballots; more than MOPS_COOP_G groups: the lanes gather themselves
                const uint64_t act = __ballot(1);
                uint64_t rem = act;
                int g = 0, G = 0;
                bool lead = false;
                while (rem != 0ull && G < kG) {
                    const int ld = __builtin_ctzll(rem);
                    const int kc = __builtin_amdgcn_readlane(cell, ld);
                    const int k0 = __builtin_amdgcn_readlane(hint0, ld);
                    const int k1 = __builtin_amdgcn_readlane(hint1, ld);
                    const bool mine = (cell == kc) & (hint0 == k0) & (hint1 == k1);
                    const uint64_t m = __ballot(mine);
                    if (mine) g = G;
                    lead |= ((int)__lane_id() == ld);
                    rem &= ~m;
                    ++G;
                }
                // the pieces are spread over the live lanes only (a dead or finished lane has left the
                // loop): at most MOPS_COOP_R per lane -- except in the hand-off kernel, which has no other
                // evaluation and takes the rest in a loop (a wave thinned by deaths, its lanes in different cells)
                const int nact = __popcll(act);
                coop = rem == 0ull && (kFillAll || G * kTilePieces <= kR * nact) &&
                       (kTileSlots >= MAXV || __ballot(c.nv > kTileSlots) == 0ull);
    #if defined(MOPS_PROF)
                // [6] cooperative wave-steps, [7] groups of the waves that were grouped in full (rem == 0);
                // [8] / [9] distinct cells / distinct (cell, hint0, hint1) per wave-step (unbounded),
                // [10] / [11] wave-steps with at most 2 of them, [12] wave-steps
                {
                    int gc = 0, gf = 0;
                    for (uint64_t r2 = act; r2 != 0ull; ++gc) {
                        const int l2 = __builtin_ctzll(r2);
                        r2 &= ~__ballot(cell == __builtin_amdgcn_readlane(cell, l2));
                    }
                    for (uint64_t r2 = act; r2 != 0ull; ++gf) {
                        const int l2 = __builtin_ctzll(r2);
                        r2 &= ~__ballot((cell == __builtin_amdgcn_readlane(cell, l2)) &
                                        (hint0 == __builtin_amdgcn_readlane(hint0, l2)) &
                                        (hint1 == __builtin_amdgcn_readlane(hint1, l2)));
                    }
                    if ((int)__lane_id() == __builtin_ctzll(act)) {
                        atomicAdd(&dev::g_prof[7], 1ull);  // regroupings
                        atomicAdd(&dev::g_prof[8], (unsigned long long)gc);
                        atomicAdd(&dev::g_prof[9], (unsigned long long)gf);
                        if (gc <= 2) atomicAdd(&dev::g_prof[10], 1ull);
                        if (gf <= 2) atomicAdd(&dev::g_prof[11], 1ull);
                        atomicAdd(&dev::g_prof[12], 1ull);
                    }
                }
    #endif
                if (coop) {
                    if (lead) {  // the group's header: {cell, nv}, then each slot's level-pair record index per field
                        const uint32_t zr = pr_zero((uint32_t)a.V, (uint32_t)a.L);
                        uint32_t r0[8], r1[8];
    #pragma unroll
                        for (int v = 0; v < 8; ++v) {
                            const bool on = v < c.nv && v < MAXV;
                            const uint32_t vid = (uint32_t)c.vid[v < MAXV ? v : 0];
                            r0[v] = (on && hint0 >= 1 && hint0 <= a.L - 1) ? pr_base((uint32_t)(hint0 - 1), vid, (uint32_t)a.V) : zr;
                            r1[v] = (on && hint1 >= 1 && hint1 <= a.L - 1) ? pr_base((uint32_t)(hint1 - 1), vid, (uint32_t)a.V) : zr;
                        }
                        uint4* hd = reinterpret_cast<uint4*>(s_hdr + g * (kTileHdr / 4));
                        hd[0] = make_uint4((uint32_t)cell, (uint32_t)c.nv, 0u, 0u);
                        hd[1] = make_uint4(r0[0], r0[1], r0[2], r0[3]);
                        hd[2] = make_uint4(r0[4], r0[5], r0[6], r0[7]);
                        hd[3] = make_uint4(r1[0], r1[1], r1[2], r1[3]);
                        hd[4] = make_uint4(r1[4], r1[5], r1[6], r1[7]);
                    }
                    dev::wave_lds_sync();  // (one wave per block: its LDS operations run in order)
                    const int np = G * kTilePieces;
                    const uint32_t* hdi = reinterpret_cast<const uint32_t*>(s_hdr);
                    const double2* cpoly2 = reinterpret_cast<const double2*>(a.cpoly);
                    const double2* cnrm2 = reinterpret_cast<const double2*>(a.cnrm);
                    const double2* cedge2 = reinterpret_cast<const double2*>(a.cedge);
                    const double2* pr0 = reinterpret_cast<const double2*>(a.f0.pr);
                    const double2* pr1 = reinterpret_cast<const double2*>(a.f1.pr);
                    // this lane's rank among the live lanes
                    const int rank = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32),
                                                                    __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
    #pragma unroll
                    for (int rr = 0; rr < kR; ++rr) {
                        const int i = rank + nact * rr;
                        if (i < np) tile_piece<MAXV>(i, hdi, cpoly2, cnrm2, cedge2, pr0, pr1, (uint32_t)a.V, s_tile);
                    }
                    if constexpr (kFillAll) {
                        for (int i = rank + nact * kR; i < np; i += nact)
                            tile_piece<MAXV>(i, hdi, cpoly2, cnrm2, cedge2, pr0, pr1, (uint32_t)a.V, s_tile);
                    }
                    dev::wave_lds_sync();
                    c.lds_n = false;  // (the tile overwrote the lane normals)
                } else if (!HAND && !c.lds_n) {  // tile mode -> lane-normal mode: each lane's normals of its cell
#pragma unroll
                    for (int k = 0; k < 3 * kNrmSlots(MAXV); ++k)
                        c.nrm[k * kTrajBlock] = a.cnrm[(int64_t)cell * kCellNrm + k];
                    c.lds_n = true;
                    dev::wave_lds_sync();
                }
                tcell = cell;
                tkey = hk | (coop ? g : 0xff);
                have_tile = coop;
                coop_prev = coop;
            } else {
                coop = coop_prev;
            }
            if (coop) tile = s_tile + (tkey & 0xff) * kTilePieces;
            if constexpr (HAND) {
                if (!(coop && hex)) {  // hand the wave over at this step (wave-uniform)
#if defined(MOPS_PROF)
                    if ((int)__lane_id() == __builtin_ctzll(__ballot(1))) {
                        atomicAdd(&dev::g_prof[14], 1ull);
                        if (!hex) atomicAdd(&dev::g_prof[15], 1ull);  // ... of them outside a hexagon
                    }
#endif
                    cell = cell_in;
                    died = -2 - (int)step;
                    break;
                }
            }
#if defined(MOPS_PROF)
            if ((int)__lane_id() == __builtin_ctzll(__ballot(1)) && coop) atomicAdd(&dev::g_prof[6], 1ull);
#endif
        }
        double hx = 0, hy = 0, hz = 0, wv = 0;
        double nx, ny, nz;
        const double alpha = PATH ? (double)step / (double)a.n_steps : 0.0;
        if (EULER) {
            bool ok = dev::eval_at<MAXV, PATH, PairGroup<PATH, EULER>::value>(hex, c, a.L, a.V, a.f0, a.f1, x, y, z, d, alpha, hint0, hint1, hx, hy, hz, wv,
                                                                              coop, tile);
            if (!ok) { died = (int)step; break; }
            MOPS_MARK(120);
            const double ax = y * hz - z * hy, ay = z * hx - x * hz, az = x * hy - y * hx;
            const double speed = dev::len3(hx, hy, hz);
            const double th = (speed * a.delta_t) / dev::dmax(1e-12, r);
            dev::rotate((unsigned)step, x, y, z, ax, ay, az, th, nx, ny, nz);
        } else {
            const double dt = (double)a.delta_t;
            const double a1 = alpha;
            // the tile's layers per field (cooperative waves; see layer_eval)
            const int th0 = (tkey >> 16) - 1, th1 = ((tkey >> 8) & 0xff) - 1;
            constexpr int GR = PairGroup<PATH, EULER>::value;
#if MOPS_RK4_LOOP
            // The four stages as one loop around a single inlined evaluation (the unrolled form inlines
            // four copies of every eval_path instantiation: ~90k instructions in the cooperative RK4
            // kernel).  The sums keep the reference's association, ((s1 + 2 s2) + 2 s3) + s4 (:959-960).
            const double a2 = PATH ? dev::dclamp(a1 + 0.5 * a.dalpha, 0.0, 1.0) : 0.0;
            const double a4 = PATH ? dev::dclamp(a1 + a.dalpha, 0.0, 1.0) : 0.0;
            double qx = x, qy = y, qz = z;
            bool ok = true;
#pragma nounroll
            for (int stg = 0; stg < 4; ++stg) {
                double sx, sy, sz, sw;
                const double as = stg == 0 ? a1 : (stg == 3 ? a4 : a2);
                ok = dev::eval_at<MAXV, PATH, GR, true, HAND>(hex, c, a.L, a.V, a.f0, a.f1, qx, qy, qz, d, as, hint0, hint1,
                                                        sx, sy, sz, sw, coop, tile, th0, th1);
                if (!ok) break;
                if (stg == 0) {
                    hx = sx; hy = sy; hz = sz; wv = sw;
                } else if (stg == 3) {
                    hx = hx + sx; hy = hy + sy; hz = hz + sz; wv = wv + sw;
                } else {
                    hx = hx + sx * 2.0; hy = hy + sy * 2.0; hz = hz + sz * 2.0; wv = wv + 2.0 * sw;
                }
                if (stg < 3) dev::advect((unsigned)step, x, y, z, sx, sy, sz, stg == 2 ? dt : dt * 0.5, qx, qy, qz);
            }
            if (!ok) { died = (int)step; break; }
            hx = hx / 6.0; hy = hy / 6.0; hz = hz / 6.0; wv = wv / 6.0;
#elif MOPS_RK4_ACC
            // The stage velocities summed as they come, in the reference's association ((s1 + 2 s2) + 2 s3) + s4
            // (:959-960): the same operations as the sum at the end, without s1..s3 live across the stages
            double sx, sy, sz, sw, qx, qy, qz;
            bool ok = dev::eval_at<MAXV, PATH, GR, true, HAND>(hex, c, a.L, a.V, a.f0, a.f1, x, y, z, d, a1, hint0, hint1,
                                                        sx, sy, sz, sw, coop, tile, th0, th1);
            if (!ok) { died = (int)step; break; }
            hx = sx; hy = sy; hz = sz; wv = sw;
            dev::advect((unsigned)step, x, y, z, sx, sy, sz, dt * 0.5, qx, qy, qz);
            const double a2 = PATH ? dev::dclamp(a1 + 0.5 * a.dalpha, 0.0, 1.0) : 0.0;
            MOPS_STAGE_FENCE();
            ok = dev::eval_at<MAXV, PATH, GR, true, HAND>(hex, c, a.L, a.V, a.f0, a.f1, qx, qy, qz, d, a2, hint0, hint1, sx, sy,
                                                   sz, sw, coop, tile, th0, th1);
            if (!ok) { died = (int)step; break; }
            hx = hx + sx * 2.0; hy = hy + sy * 2.0; hz = hz + sz * 2.0; wv = wv + 2.0 * sw;
            dev::advect((unsigned)step, x, y, z, sx, sy, sz, dt * 0.5, qx, qy, qz);
            MOPS_STAGE_FENCE();
            ok = dev::eval_at<MAXV, PATH, GR, true, HAND>(hex, c, a.L, a.V, a.f0, a.f1, qx, qy, qz, d, a2, hint0, hint1, sx, sy,
                                                   sz, sw, coop, tile, th0, th1);
            if (!ok) { died = (int)step; break; }
            hx = hx + sx * 2.0; hy = hy + sy * 2.0; hz = hz + sz * 2.0; wv = wv + 2.0 * sw;
            dev::advect((unsigned)step, x, y, z, sx, sy, sz, dt, qx, qy, qz);
            const double a4 = PATH ? dev::dclamp(a1 + a.dalpha, 0.0, 1.0) : 0.0;
            MOPS_STAGE_FENCE();
            ok = dev::eval_at<MAXV, PATH, GR, true, HAND>(hex, c, a.L, a.V, a.f0, a.f1, qx, qy, qz, d, a4, hint0, hint1, sx, sy,
                                                   sz, sw, coop, tile, th0, th1);
            if (!ok) { died = (int)step; break; }
            hx = (hx + sx) / 6.0; hy = (hy + sy) / 6.0; hz = (hz + sz) / 6.0; wv = (wv + sw) / 6.0;
#else
            double s1x, s1y, s1z, s1w, s2x, s2y, s2z, s2w, s3x, s3y, s3z, s3w, s4x, s4y, s4z, s4w;
            double qx, qy, qz;
            bool ok = dev::eval_at<MAXV, PATH, GR, true, HAND>(hex, c, a.L, a.V, a.f0, a.f1, x, y, z, d, a1, hint0, hint1,
                                                        s1x, s1y, s1z, s1w, coop, tile, th0, th1);
            if (!ok) { died = (int)step; break; }
            dev::advect((unsigned)step, x, y, z, s1x, s1y, s1z, dt * 0.5, qx, qy, qz);
            const double a2 = PATH ? dev::dclamp(a1 + 0.5 * a.dalpha, 0.0, 1.0) : 0.0;
            ok = dev::eval_at<MAXV, PATH, GR, true, HAND>(hex, c, a.L, a.V, a.f0, a.f1, qx, qy, qz, d, a2, hint0, hint1, s2x,
                                                   s2y, s2z, s2w, coop, tile, th0, th1);
            if (!ok) { died = (int)step; break; }
            dev::advect((unsigned)step, x, y, z, s2x, s2y, s2z, dt * 0.5, qx, qy, qz);
            ok = dev::eval_at<MAXV, PATH, GR, true, HAND>(hex, c, a.L, a.V, a.f0, a.f1, qx, qy, qz, d, a2, hint0, hint1, s3x,
                                                   s3y, s3z, s3w, coop, tile, th0, th1);
            if (!ok) { died = (int)step; break; }
            dev::advect((unsigned)step, x, y, z, s3x, s3y, s3z, dt, qx, qy, qz);
            const double a4 = PATH ? dev::dclamp(a1 + a.dalpha, 0.0, 1.0) : 0.0;
            ok = dev::eval_at<MAXV, PATH, GR, true, HAND>(hex, c, a.L, a.V, a.f0, a.f1, qx, qy, qz, d, a4, hint0, hint1, s4x,
                                                   s4y, s4z, s4w, coop, tile, th0, th1);
            if (!ok) { died = (int)step; break; }
            // (s1 + 2 s2 + 2 s3 + s4) / 6 -- cy::Vec3 operator order (:959-960)
            hx = (((s1x + s2x * 2.0) + s3x * 2.0) + s4x) / 6.0;
            hy = (((s1y + s2y * 2.0) + s3y * 2.0) + s4y) / 6.0;
            hz = (((s1z + s2z * 2.0) + s3z * 2.0) + s4z) / 6.0;
            wv = (s1w + 2.0 * s2w + 2.0 * s3w + s4w) / 6.0;
#endif
            const double tx = x + hx * dt, ty = y + hy * dt, tz = z + hz * dt;
            const double tl = dev::len3(tx, ty, tz);
            if (tl > 1e-12) {
                dev::xdiv_norm3(tx, ty, tz, tl, nx, ny, nz);
                nx *= r; ny *= r; nz *= r;
            }
            else { nx = x; ny = y; nz = z; }
        }
        MOPS_MARK(130);
        // vertical update (:977-986)
        const double old_depth = (double)dep;
        double nd = old_depth - wv * (double)a.delta_t;
        nd = dev::dmax(0.0, nd);
        const double r_new = dev::dmax(1.0, r + wv * (double)a.delta_t);
        dep = (float)nd;
        const double nl = dev::len3(nx, ny, nz);
        if (nl > 1e-12) {
            dev::xdiv_norm3(nx, ny, nz, nl, nx, ny, nz);
            nx *= r_new; ny *= r_new; nz *= r_new;
        }
        MOPS_MARK(140);
        if (step == 0) {  // first_vel (:988-991)
            a.rec[3 * a.rec_stride + pid] = hx;
            a.rec[4 * a.rec_stride + pid] = hy;
            a.rec[5 * a.rec_stride + pid] = hz;
        }
        x = nx; y = ny; z = nz;
        if (step == rec_next) {  // (step + 1) % rec_period == 0, record k = (step + 1) / rec_period - 1
            const int64_t k = rec_k;
            rec_next += a.rec_period;
            ++rec_k;
            MOPS_MARK(150);
            if (k < a.K) {
                double* rk = a.rec + k * 6 * a.rec_stride;
                rk[0 * a.rec_stride + pid] = x;
                rk[1 * a.rec_stride + pid] = y;
                rk[2 * a.rec_stride + pid] = z;
                rk[3 * a.rec_stride + pid] = hx;
                rk[4 * a.rec_stride + pid] = hy;
                rk[5 * a.rec_stride + pid] = hz;
            }
        }
    }
    a.px[pid] = x; a.py[pid] = y; a.pz[pid] = z;
    a.depth[pid] = dep;
    a.cell[pid] = cell;
    if constexpr (HAND) {
        if (died != -1) a.death[pid] = died;  // (-2 - step at a hand-off)
    } else {
        if (died >= 0 || resumed) a.death[pid] = died;  // (resumed: -1 again unless it died)
    }
    // slots never sampled: after a death, and past the last record step of a run whose
    // record period does not fill all K slots (streamline recordT % deltaT != 0)
    if constexpr (HAND) {
        if (died >= 0 || (a.step_end == a.n_steps && died == -1))
            dev::clear_records(a.rec, a.rec_stride, pid, (rec_k == 0 && rec0) ? 1 : rec_k, a.K);
    } else {
        if (died >= 0 || a.step_end == a.n_steps) dev::clear_records(a.rec, a.rec_stride, pid, (rec_k == 0 && rec0) ? 1 : rec_k, a.K);
    }
}

// the neighbour-table test against the walk it short-cuts (mops_selftest_walk): bit 0 = dev::nbr_stay kept
// the cell, bit 1 = dev::walk kept it, bits 8.. = the stay-ball radius nbr_stay set, in metres (clamped)
__global__ void selftest_walk_kernel(int64_t n, const double* __restrict__ pts, const int* __restrict__ cells,
                                     const int* __restrict__ cellrec, const double4* __restrict__ cxyz,
                                     const uint4* __restrict__ nbr, int C, int* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int cell = cells[i];
    if (cell < 0 || cell >= C) { out[i] = -1; return; }
    const double x = pts[3 * i], y = pts[3 * i + 1], z = pts[3 * i + 2];
    dev::Cell<7> c;
    c.nv = cellrec[(int64_t)cell * (((1 + 2 * 7) + 3) / 4 * 4)];
    c.rs2 = 0.0;
    const bool a = dev::nbr_stay<7, false>(c, cell, x, y, z, nbr);
    const double rad = a ? sqrt(c.rs2) : 0.0;
    const bool b = dev::walk<7, false>(c, cell, x, y, z, cellrec, cxyz, C) == cell;
    const int rq = (int)fmin(rad, 4.0e6);  // (< 2^22)
    out[i] = (a ? 1 : 0) | (b ? 2 : 0) | (rq << 8);
}

// exact math helpers against the library (mops_selftest_math)
__global__ void selftest_math_kernel(int64_t n, const double* __restrict__ x, double* __restrict__ out, int op) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (op == 2) {  // x = n vectors (3 doubles each); out = 3 fast + 3 library quotients by their length
        const double a0 = x[3 * i], a1 = x[3 * i + 1], a2 = x[3 * i + 2];
        const double b = dev::len3(a0, a1, a2);
        double q0 = 0.0, q1 = 0.0, q2 = 0.0;
        if (b > 1e-12) dev::xdiv_norm3(a0, a1, a2, b, q0, q1, q2);
        out[6 * i] = q0; out[6 * i + 1] = q1; out[6 * i + 2] = q2;
        out[6 * i + 3] = b > 1e-12 ? a0 / b : 0.0;
        out[6 * i + 4] = b > 1e-12 ? a1 / b : 0.0;
        out[6 * i + 5] = b > 1e-12 ? a2 / b : 0.0;
        return;
    }
    const double v = x[i];
    if (op == 0) {
        out[2 * i] = dev::xsqrt(v);
        out[2 * i + 1] = sqrt(v);
    } else {
        const double ls = sin(v), lc = cos(v);
        double s = ls, c = lc;
        if (fabs(v) < 0.78) dev::sincos_small(v, s, c, (unsigned)i);
        out[4 * i] = s; out[4 * i + 1] = ls; out[4 * i + 2] = c; out[4 * i + 3] = lc;
    }
}

// ===========================================================================
// output assembly: FinalizeTrajectoryLines[WithAttrs] + RemoveNaN
// ===========================================================================
// xyz -> {lat, lon (deg), r, |v|} per line point (GeoConverter::convertXYZToLatLonDegree,
// VTKFileManager.hpp:352-395) -- the streaming half of the output writers
__global__ void lines_geo_kernel(int64_t m, const double* __restrict__ pts, const double* __restrict__ vel,
                                 double* __restrict__ geo) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= m) return;
    const double x = pts[3 * i], y = pts[3 * i + 1], z = pts[3 * i + 2];
    const double r = sqrt(x * x + y * y + z * z);
    const double theta = asin(z / r), phi = atan2(y, x);
    double vm = 0.0;
    if (vel) {
        const double vx = vel[3 * i], vy = vel[3 * i + 1], vz = vel[3 * i + 2];
        vm = sqrt(vx * vx + vy * vy + vz * vz);
    }
    double4 o;
    o.x = theta * (180.0 / M_PI); o.y = phi * (180.0 / M_PI); o.z = r; o.w = vm;
    reinterpret_cast<double4*>(geo)[i] = o;
}

__device__ __forceinline__ bool finite3(double a, double b, double c) { return isfinite(a) && isfinite(b) && isfinite(c); }

// One thread per line.  Uniform lines (off == NULL): line i is points [i*P, (i+1)*P); ragged
// lines: [off[i], off[i+1]) -- the reference's per-line vectors packed back to back.  An empty
// line is left alone (the reference drops it, TrajectoryCommon.h:84-86: the host re-indexes).
// Uniform lines written through a slot -> line map (line != NULL, a particle part's assembly into the
// full outputs): thread i cleans line line[i], the one its slot's assembly wrote.
__global__ void remove_nan_kernel(int64_t n, int64_t P, const int64_t* __restrict__ off, double* pts, double* vel,
                                  double* tmp, double* sal, double* last, const int32_t* __restrict__ line = nullptr) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    if (!off && line) i = line[i];
    const int64_t b = off ? off[i] : i * P;
    if (off) P = off[i + 1] - b;
    if (P <= 0) return;
    double* pp = pts + 3 * b;
    double* vv = vel ? vel + 3 * b : nullptr;
    double* tt = tmp ? tmp + b : nullptr;
    double* ss = sal ? sal + b : nullptr;
    int64_t k = 0;
    for (; k < P; ++k)
        if (!finite3(pp[3 * k], pp[3 * k + 1], pp[3 * k + 2])) break;
    if (k < P) {
        const int64_t src = (k == 0) ? 0 : k - 1;
        const double lx = pp[3 * src], ly = pp[3 * src + 1], lz = pp[3 * src + 2];
        const double lt = tt ? tt[src] : 0.0, ls = ss ? ss[src] : 0.0;
        const int64_t j0 = (k == 0) ? 0 : k - 1;
        for (int64_t j = j0; j < P; ++j) {
            if (j >= k || k == 0) {
                pp[3 * j] = lx; pp[3 * j + 1] = ly; pp[3 * j + 2] = lz;
                if (tt) tt[j] = lt;
                if (ss) ss[j] = ls;
            }
            if (vv) { vv[3 * j] = 0.0; vv[3 * j + 1] = 0.0; vv[3 * j + 2] = 0.0; }
        }
    }
    if (last) {
        last[3 * i] = pp[3 * (P - 1)];
        last[3 * i + 1] = pp[3 * (P - 1) + 1];
        last[3 * i + 2] = pp[3 * (P - 1) + 2];
    }
}

// Records [K][6][stride] (slot-major) -> lines [n][P] (line-major): a
// transpose, staged through LDS in tiles of 32 slots x 8 records so that both
// the record reads (32 consecutive slots) and the line writes (8 records x 3
// doubles contiguous per line) coalesce.  Line of slot i = line ? line[i] : i.
constexpr int kAsmSlots = 32, kAsmRecs = 8;
__global__ void __launch_bounds__(256) assemble_kernel(int64_t n, int64_t K, const double* __restrict__ seeds,
                                                       const double* __restrict__ rec, int64_t stride, int pathline,
                                                       const int32_t* __restrict__ line, double* __restrict__ pts,
                                                       double* __restrict__ vel, double* __restrict__ tmp,
                                                       double* __restrict__ sal) {
    __shared__ double tile[kAsmRecs][6][kAsmSlots + 1];
    __shared__ int64_t row[kAsmSlots];
    const int t = threadIdx.x;
    const int64_t s0 = (int64_t)blockIdx.x * kAsmSlots;
    const int ns = (int)((n - s0) < kAsmSlots ? (n - s0) : kAsmSlots);
    const int64_t P = K + 1;
    if (t < ns) {
        const int64_t r = line ? (int64_t)line[s0 + t] : s0 + t;
        row[t] = r;
        double* pp = pts + 3 * r * P;  // points[0] = seed
        pp[0] = seeds[3 * (s0 + t)]; pp[1] = seeds[3 * (s0 + t) + 1]; pp[2] = seeds[3 * (s0 + t) + 2];
        if (vel) { double* vv = vel + 3 * (r * P + K); vv[0] = 0.0; vv[1] = 0.0; vv[2] = 0.0; }  // appended zero
        if (tmp) tmp[r * P + K] = 0.0;
        if (sal) sal[r * P + K] = 0.0;
    }
    for (int64_t k0 = 0; k0 < K; k0 += kAsmRecs) {
        const int nk = (int)((K - k0) < kAsmRecs ? (K - k0) : kAsmRecs);
        __syncthreads();  // previous chunk consumed (and row[] written)
        for (int e = t; e < kAsmRecs * 6 * kAsmSlots; e += blockDim.x) {
            const int i = e % kAsmSlots, c = (e / kAsmSlots) % 6, kk = e / (kAsmSlots * 6);
            if (i < ns && kk < nk) tile[kk][c][i] = rec[(k0 + kk) * 6 * stride + c * stride + s0 + i];
        }
        __syncthreads();
        for (int e = t; e < kAsmSlots * kAsmRecs * 3; e += blockDim.x) {
            const int i = e / (kAsmRecs * 3), off = e % (kAsmRecs * 3), kk = off / 3, c = off % 3;
            if (i < ns && kk < nk) {
                const int64_t r = row[i];
                pts[3 * (r * P + k0 + kk + 1) + c] = tile[kk][c][i];
                if (vel) vel[3 * (r * P + k0 + kk) + c] = tile[kk][3 + c][i];
            }
        }
        if (tmp || sal) {
            for (int e = t; e < kAsmSlots * kAsmRecs; e += blockDim.x) {
                const int i = e / kAsmRecs, kk = e % kAsmRecs;
                if (i < ns && kk < nk) {
                    const int64_t r = row[i];
                    if (tmp) tmp[r * P + k0 + kk] = pathline ? tile[kk][3][i] : 0.0;
                    if (sal) sal[r * P + k0 + kk] = pathline ? tile[kk][4][i] : 0.0;
                }
            }
        }
    }
}

// Assembly and NaN cleanup in one pass when a line's K records fit the block's LDS tile (K <=
// kAsmFull: every record period of a day's run at 1 h records): the whole [K][6][32-slot] slab
// plus the seeds is staged, each line's first non-finite point found there, and the cleaned
// line -- RemoveNaNTrajectoriesAndReindex's padding with the last finite point, zeroed velocity
// from the point before it, temperature/salinity held (TrajectoryCommon.h:92-121) -- written
// once, with consecutive threads on consecutive doubles of a line (whole 600-B point runs at K =
// 24 instead of 192-B chunks), saving remove_nan_kernel's second, strided pass over the lines.
constexpr int kAsmFull = 24;
#ifndef MOPS_ASM_V2
// 16-B record reads (even stride, full blocks) and streaming (non-temporal) line stores: config 3's per-pair
// assembly 9.71 -> 8.46 ms, its 7-pair chain 3620 -> 3610 ms (3 interleaved rounds,
// profiles/r05/ab/assembly_v2.txt)
#define MOPS_ASM_V2 1
#endif
template <typename T>
__device__ __forceinline__ void asm_store(T* p, T v) {
#if MOPS_ASM_V2
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}
__global__ void __launch_bounds__(256) assemble_clean_kernel(int64_t n, int K, const double* __restrict__ seeds,
                                                             const double* __restrict__ rec, int64_t stride,
                                                             int pathline, const int32_t* __restrict__ line,
                                                             double* __restrict__ pts, double* __restrict__ vel,
                                                             double* __restrict__ tmp, double* __restrict__ sal,
                                                             double* __restrict__ last) {
    __shared__ double tile[kAsmFull][6][kAsmSlots + 1];
    __shared__ double seed[kAsmSlots][3];
    __shared__ int64_t row[kAsmSlots];
    __shared__ int cut[kAsmSlots];
    const int t = threadIdx.x;
    const int64_t s0 = (int64_t)blockIdx.x * kAsmSlots;
    const int ns = (int)((n - s0) < kAsmSlots ? (n - s0) : kAsmSlots);
    const int P = K + 1;
#if MOPS_ASM_V2
    // (block-uniform) 16-B pieces, 2 slots per load: needs an even stride and a 16-B aligned slab (a caller's
    // finalize_range passes records + 8 lo for any lo)
    if (ns == kAsmSlots && (stride & 1) == 0 && (reinterpret_cast<uintptr_t>(rec) & 15) == 0) {
        for (int e = t; e < K * 6 * (kAsmSlots / 2); e += blockDim.x) {
            const int i2 = e % (kAsmSlots / 2), c = (e / (kAsmSlots / 2)) % 6, kk = e / ((kAsmSlots / 2) * 6);
            const double2 v = *reinterpret_cast<const double2*>(rec + kk * 6 * stride + c * stride + s0 + 2 * i2);
            tile[kk][c][2 * i2] = v.x;
            tile[kk][c][2 * i2 + 1] = v.y;
        }
    } else
#endif
    for (int e = t; e < K * 6 * kAsmSlots; e += blockDim.x) {
        const int i = e % kAsmSlots, c = (e / kAsmSlots) % 6, kk = e / (kAsmSlots * 6);
        if (i < ns) tile[kk][c][i] = rec[kk * 6 * stride + c * stride + s0 + i];
    }
    for (int e = t; e < 3 * kAsmSlots; e += blockDim.x)
        if (e / 3 < ns) seed[e / 3][e % 3] = seeds[3 * s0 + e];
    if (t < ns) row[t] = line ? (int64_t)line[s0 + t] : s0 + t;
    __syncthreads();
    // original point j of line i: seed, then the records' positions
    auto point = [&](int i, int j, int c) -> double { return j == 0 ? seed[i][c] : tile[j - 1][c][i]; };
    if (t < ns) {
        int k = 0;
        for (; k < P; ++k)
            if (!finite3(point(t, k, 0), point(t, k, 1), point(t, k, 2))) break;
        cut[t] = k;
    }
    __syncthreads();
    for (int e = t; e < ns * P * 3; e += blockDim.x) {  // points (and velocities)
        const int i = e / (P * 3), off = e - i * (P * 3), j = off / 3, c = off - j * 3, k = cut[i];
        const int64_t o = 3 * row[i] * P + off;
        asm_store(pts + o, (k < P && (k == 0 || j >= k)) ? point(i, k == 0 ? 0 : k - 1, c) : point(i, j, c));
        if (vel) asm_store(vel + o, (j == K || (k < P && (k == 0 || j >= k - 1))) ? 0.0 : tile[j][3 + c][i]);
    }
    if (tmp || sal) {
        for (int e = t; e < ns * P; e += blockDim.x) {
            const int i = e / P, j = e - i * P, k = cut[i];
            const int src = (k < P && (k == 0 || j >= k)) ? (k == 0 ? 0 : k - 1) : j;  // held value's index
            const int64_t o = row[i] * P + j;
            if (tmp) asm_store(tmp + o, (pathline && src < K) ? tile[src][3][i] : 0.0);
            if (sal) asm_store(sal + o, (pathline && src < K) ? tile[src][4][i] : 0.0);
        }
    }
    if (last) {
        for (int e = t; e < ns * 3; e += blockDim.x) {
            const int i = e / 3, c = e - i * 3, k = cut[i];
            asm_store(last + 3 * row[i] + c, (k < P) ? point(i, k == 0 ? 0 : k - 1, c) : point(i, K, c));  // line order
        }
    }
}

// The cleaned last point of every line alone -- assemble_clean_kernel's `last` (the last finite point
// before the first non-finite one, the seed when the seed itself is not finite, else the final record;
// RemoveNaNTrajectoriesAndReindex, TrajectoryCommon.h:92-121) -- without assembling the lines: a chained
// pair's next seeds, so the full assembly can run beside the next pair (mops_traj_last_points).
// One lane per slot; record k's x/y/z rows are read coalesced across the slots, stopping at the cut.
__global__ void __launch_bounds__(256) last_point_kernel(int64_t n, int K, const double* __restrict__ seeds,
                                                         const double* __restrict__ rec, int64_t stride,
                                                         const int32_t* __restrict__ line, double* __restrict__ last) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double lx = seeds[3 * i], ly = seeds[3 * i + 1], lz = seeds[3 * i + 2];
    if (finite3(lx, ly, lz)) {
        for (int k = 0; k < K; ++k) {
            const double* r = rec + (int64_t)k * 6 * stride + i;
            const double x = r[0], y = r[stride], z = r[2 * stride];
            if (!finite3(x, y, z)) break;
            lx = x; ly = y; lz = z;
        }
    }
    const int64_t o = line ? (int64_t)line[i] : i;
    last[3 * o] = lx;
    last[3 * o + 1] = ly;
    last[3 * o + 2] = lz;
}

// ===========================================================================
// derived-field preprocessing (once per snapshot)
// ===========================================================================

// MPASOSolution::calcCellCenterZtop (MPASOSolution.cpp:535-618): zTop from layerThickness and
// bottomDepth (bottom up), or from the surface height (top down), or from 0; each row's
// recurrence in the reference's order, with the block's rows staged through LDS: kZtCells consecutive cells are
// one contiguous [kZtCells][L] slab of thick (and of ztop), so it is read and written with
// coalesced wave-wide accesses; one thread per cell runs its row's recurrence in LDS, in the
// reference's order (a per-cell thread streaming its own row made every wave access 64 rows L
// doubles apart: 0.6 TB/s on an oRRS18to6-class snapshot).
constexpr int kZtCells = 64;
__global__ void __launch_bounds__(256) cell_ztop_tiled_kernel(int64_t C, int L, const double* __restrict__ thick,
                                                              const double* __restrict__ bottom,
                                                              const double* __restrict__ ssh,
                                                              double* __restrict__ ztop) {
    extern __shared__ double zt_tile[];  // [kZtCells * L]
    const int64_t c0 = (int64_t)blockIdx.x * kZtCells;
    const int nc = (int)((C - c0) < kZtCells ? (C - c0) : kZtCells);
    const int64_t base = c0 * L;
    const int n = nc * L;
    for (int i = threadIdx.x; i < n; i += blockDim.x) zt_tile[i] = thick[base + i];
    __syncthreads();
    if ((int)threadIdx.x < nc) {
        double* row = zt_tile + threadIdx.x * L;
        const int64_t i = c0 + threadIdx.x;
        if (bottom) {
            double z = -bottom[i];
            for (int k = L - 1; k >= 0; --k) { z += row[k]; row[k] = z * 1.0; }
        } else if (ssh) {
            double z = ssh[i];
            double tp = row[0];  // thick[j-1] for j = 1, read before row[0] is overwritten
            row[0] = z * 1.0;
            for (int j = 1; j < L; ++j) { const double t = row[j]; z -= tp; row[j] = z * 1.0; tp = t; }
        } else {
            double prev = 0.0;
            double tp = row[0];
            row[0] = 0.0;
            for (int j = 1; j < L; ++j) { const double t = row[j]; prev = prev - tp; row[j] = prev * 1.0; tp = t; }
        }
    }
    __syncthreads();
    for (int i = threadIdx.x; i < n; i += blockDim.x) ztop[base + i] = zt_tile[i];
}

// CalcCellCenterVelocityByZM + GeoConverter::convertENUVelocityToXYZ (Uup = 0)
__global__ void center_vel_zm_kernel(int64_t C, int L, const double4* cxyz, const double* zonal, const double* mer,
                                     double* out) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= C * L) return;
    const int64_t c = idx / L;
    const double4 p = cxyz[c];
    const double uz = zonal[idx], um = mer[idx], uu = 0.0;
    double* o = out + 3 * idx;
    if (p.x == 0.0 && p.y == 0.0) { o[0] = 0.0; o[1] = 0.0; o[2] = uu; return; }
    const double Rxy = sqrt(p.x * p.x + p.y * p.y);
    const double Rxyz = sqrt(p.x * p.x + p.y * p.y + p.z * p.z);
    const double slon = p.y / Rxy, clon = p.x / Rxy, slat = p.z / Rxyz, clat = Rxy / Rxyz;
    o[0] = -slon * uz - slat * clon * um + clon * clat * uu;
    o[1] = clon * uz - slat * slon * um + slon * clat * uu;
    o[2] = clat * um + slat * uu;
}

// ---------------------------------------------------------------------------
// RBF reconstruction of the cell-centre velocity from edge normals
// (TBBBackend::CalcCellCenterVelocity, MPASOSolutionTBB.cpp:131-245, with
// Interpolator::mpas_rbf_interp_func_3D_plane_vec_const_dir_comp_coeffs and
// gauss_elimination_fixed, Interpolation.hpp:167-340).  The reference solves
// the same two 7x7 systems for every (cell, layer); they depend on the cell's
// geometry only, so the engine solves them once per cell when the mesh's edges
// are uploaded (rbf_coef_kernel, same operations in the same order) and each
// snapshot's derivation is the reference's final 7-term sums per (cell,
// layer) (rbf_apply_kernel).  Quirks kept: pointCount is always
// MAX_VERTEX_NUM = 7 (absent edges are zero points with zero unit vectors,
// which makes the system singular -- NaN -- for every cell with fewer than 7
// edges), alpha is forced to 1 and the right-hand side evaluates the RBF at 1.
// ---------------------------------------------------------------------------
constexpr int kRbfN = 7;

__device__ __forceinline__ void rbf_gauss7(double (&A)[8][8], double (&b)[8], double (&x)[8]) {
    int pivot[8];
#pragma unroll
    for (int i = 0; i < kRbfN; i++) pivot[i] = i;
    for (int j = 0; j < kRbfN - 1; ++j) {
        int maxRow = j;
        for (int i = j + 1; i < kRbfN; ++i)
            if (fabs(A[pivot[i]][j]) > fabs(A[pivot[maxRow]][j])) maxRow = i;
        const int tmp = pivot[j]; pivot[j] = pivot[maxRow]; pivot[maxRow] = tmp;
        for (int i = j + 1; i < kRbfN; ++i) {
            const double factor = A[pivot[i]][j] / A[pivot[j]][j];
            A[pivot[i]][j] = factor;
            for (int k = j + 1; k < kRbfN; ++k) A[pivot[i]][k] -= factor * A[pivot[j]][k];
            b[pivot[i]] -= factor * b[pivot[j]];
        }
    }
    x[kRbfN - 1] = b[pivot[kRbfN - 1]] / A[pivot[kRbfN - 1]][kRbfN - 1];
    for (int i = kRbfN - 2; i >= 0; --i) {
        double sum = 0.0;
        for (int j = i + 1; j < kRbfN; ++j) sum += A[pivot[i]][j] * x[j];
        x[i] = (b[pivot[i]] - sum) / A[pivot[i]][i];
    }
}

// one thread per cell: coef [C][7][3] and the 7 edge ids (-1 = the slot's velocity is 0)
__global__ void __launch_bounds__(64) rbf_coef_kernel(int64_t C, int rec_ints, const int* __restrict__ cellrec,
                                                      const int* __restrict__ eoc, const int2* __restrict__ coe,
                                                      const double4* __restrict__ exyz,
                                                      const double4* __restrict__ cxyz, double* __restrict__ coef,
                                                      int* __restrict__ slot_edge) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const double4 p = cxyz[c];
    const int nv = cellrec[c * rec_ints];
    const double pl = sqrt(p.x * p.x + p.y * p.y + p.z * p.z);
    const double ux = p.x / pl, uy = p.y / pl, uz = p.z / pl;                          // up
    double ex = 0.0 * uz - 1.0 * uy, ey = 1.0 * ux - 0.0 * uz, ez = 0.0 * uy - 0.0 * ux;  // (0,0,1) x up
    if (sqrt(ex * ex + ey * ey + ez * ez) < 1e-6) {
        ex = 1.0 * uz - 0.0 * uy; ey = 0.0 * ux - 0.0 * uz; ez = 0.0 * uy - 1.0 * ux;      // (0,1,0) x up
    }
    const double el = sqrt(ex * ex + ey * ey + ez * ez);
    ex = ex / el; ey = ey / el; ez = ez / el;
    const double nx = uy * ez - uz * ey, ny = uz * ex - ux * ez, nz = ux * ey - uy * ex;  // up x east
    const double pb[2][3] = {{ex, ey, ez}, {nx, ny, nz}};
    double ps[8][2], pu[8][2];
    int sl[8];
#pragma unroll
    for (int s = 0; s < kRbfN; ++s) {
        double e0 = 0.0, e1 = 0.0, e2 = 0.0, n0 = 0.0, n1 = 0.0, n2 = 0.0;
        int e = (s < nv) ? eoc[c * kRbfN + s] : -1;
        if (e >= 0) {
            const double4 ep = exyz[e];
            e0 = ep.x; e1 = ep.y; e2 = ep.z;
            const int2 ce = coe[e];  // 0-based, -1 = none (the reference's SIZE_MAX)
            const uint64_t c0 = (uint64_t)(int64_t)ce.x, c1 = (uint64_t)(int64_t)ce.y;
            const uint64_t lo = c0 < c1 ? c0 : c1, hi = c0 > c1 ? c0 : c1;
            double vx, vy, vz;
            const double4 a = cxyz[lo];
            if (hi > (uint64_t)C) {
                vx = ep.x - a.x; vy = ep.y - a.y; vz = ep.z - a.z;
            } else {
                const double4 b = cxyz[hi];
                vx = b.x - a.x; vy = b.y - a.y; vz = b.z - a.z;
            }
            const double l = sqrt(vx * vx + vy * vy + vz * vz);
            if (l == 0.0) {
                e = -1;  // skipped: the slot keeps its edge centre, zero unit vector and zero velocity
            } else {
                n0 = vx / l; n1 = vy / l; n2 = vz / l;
            }
            // (the reference records the edge centre before the length test)
        }
        sl[s] = e;
        ps[s][0] = e0 * pb[0][0] + e1 * pb[0][1] + e2 * pb[0][2];
        ps[s][1] = e0 * pb[1][0] + e1 * pb[1][1] + e2 * pb[1][2];
        pu[s][0] = n0 * pb[0][0] + n1 * pb[0][1] + n2 * pb[0][2];
        pu[s][1] = n0 * pb[1][0] + n1 * pb[1][1] + n2 * pb[1][2];
    }
    double A[8][8], rhs[8][2];
    const double rvd = 1.0 / sqrt(1.0 + 1.0);  // evaluate_rbf(1.0)
    for (int j = 0; j < kRbfN; ++j) {
        for (int i = j; i < kRbfN; ++i) {
            double r2 = 0.0;
            double diff = ps[i][0] - ps[j][0];
            r2 += diff * diff;
            diff = ps[i][1] - ps[j][1];
            r2 += diff * diff;
            r2 /= (1.0 * 1.0);
            const double rv = 1.0 / sqrt(1.0 + r2);
            const double dp = pu[i][0] * pu[j][0] + pu[i][1] * pu[j][1];
            A[i][j] = rv * dp;
            A[j][i] = A[i][j];
        }
        rhs[j][0] = rvd * pu[j][0];
        rhs[j][1] = rvd * pu[j][1];
    }
    double Ac[8][8], b[8], x1[8], x2[8];
    for (int i = 0; i < kRbfN; ++i)
        for (int j = 0; j < kRbfN; ++j) Ac[i][j] = A[i][j];
    for (int i = 0; i < kRbfN; ++i) b[i] = rhs[i][0];
    rbf_gauss7(Ac, b, x1);
    for (int i = 0; i < kRbfN; ++i)
        for (int j = 0; j < kRbfN; ++j) Ac[i][j] = A[i][j];
    for (int i = 0; i < kRbfN; ++i) b[i] = rhs[i][1];
    rbf_gauss7(Ac, b, x2);
    for (int i = 0; i < kRbfN; ++i) {
        double* o = coef + (c * kRbfN + i) * 3;
        o[0] = pb[0][0] * x1[i] + pb[1][0] * x2[i];
        o[1] = pb[0][1] * x1[i] + pb[1][1] * x2[i];
        o[2] = pb[0][2] * x1[i] + pb[1][2] * x2[i];
        slot_edge[c * kRbfN + i] = sl[i];
    }
}

// one thread per (cell, layer): the reference's 7-term sums (:234-243); a slot without an edge
// (or with a zero-length normal) contributes coef * 0.0, as in the reference
__global__ void rbf_apply_kernel(int64_t C, int L, const double* __restrict__ coef, const int* __restrict__ slot_edge,
                                 const double* __restrict__ normal_vel, double* __restrict__ out) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= C * L) return;
    const int64_t c = idx / L;
    const int k = (int)(idx - c * L);
    double xv = 0.0, yv = 0.0, zv = 0.0;
#pragma unroll
    for (int s = 0; s < kRbfN; ++s) {
        const int e = slot_edge[c * kRbfN + s];
        const double nv = (e >= 0) ? normal_vel[(int64_t)e * L + k] : 0.0;
        const double* q = coef + (c * kRbfN + s) * 3;
        xv += q[0] * nv;
        yv += q[1] * nv;
        zv += q[2] * nv;
    }
    double* o = out + 3 * idx;
    o[0] = xv; o[1] = yv; o[2] = zv;
}

// CalcCellVertexZtop / CenterToVertex / VertexVelocity / VertexVertVelocity
// (MPASOSolutionTBB.cpp:9-106, 270-366): barycentric of the 3 cellsOnVertex.  The weights of each
// vertex in its three cellsOnVertex centres are computed once per mesh (the reference recomputes
// them per (vertex, level); same operations, so bit-identical): {u, v, w, 1}, or {0, 0, 0, 0}
// for a boundary vertex (a missing cell, quirk Q10); cell_to_vertex_bary_kernel then applies them
// to every level.
__global__ void vertex_bary_kernel(int64_t V, const int* __restrict__ cov, const double4* __restrict__ cxyz,
                                   const double4* __restrict__ vxyz, double4* __restrict__ bary) {
    const int64_t vid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (vid >= V) return;
    const int c0 = cov[3 * vid], c1 = cov[3 * vid + 1], c2 = cov[3 * vid + 2];
    double4 b = make_double4(0.0, 0.0, 0.0, 0.0);
    if (c0 >= 0 && c1 >= 0 && c2 >= 0) {
        const double4 p = vxyz[vid], A = cxyz[c0], B = cxyz[c1], Cc = cxyz[c2];
        const double v0x = B.x - A.x, v0y = B.y - A.y, v0z = B.z - A.z;
        const double v1x = Cc.x - A.x, v1y = Cc.y - A.y, v1z = Cc.z - A.z;
        const double v2x = p.x - A.x, v2y = p.y - A.y, v2z = p.z - A.z;
        const double d00 = v0x * v0x + v0y * v0y + v0z * v0z;
        const double d01 = v0x * v1x + v0y * v1y + v0z * v1z;
        const double d11 = v1x * v1x + v1y * v1y + v1z * v1z;
        const double d20 = v2x * v0x + v2y * v0y + v2z * v0z;
        const double d21 = v2x * v1x + v2y * v1y + v2z * v1z;
        const double den = d00 * d11 - d01 * d01;
        const double v = (d11 * d20 - d01 * d21) / den;
        const double w = (d00 * d21 - d01 * d20) / den;
        const double u = 1.0 - v - w;
        b = make_double4(u, v, w, 1.0);
    }
    bary[vid] = b;
}

template <int DIM>
__global__ void cell_to_vertex_bary_kernel(int64_t V, int Lt, const int* __restrict__ cov,
                                           const double4* __restrict__ bary, const double* __restrict__ src,
                                           double* __restrict__ dst, int clamp_neg,
                                           const int* __restrict__ vrow = nullptr) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= V * Lt) return;
    const int64_t vid = idx / Lt;
    const int k = (int)(idx - vid * Lt);
    const double4 b = bary[vid];
    double out[DIM];
#pragma unroll
    for (int d = 0; d < DIM; ++d) out[d] = 0.0;
    if (b.w != 0.0) {
        const int c0 = cov[3 * vid], c1 = cov[3 * vid + 1], c2 = cov[3 * vid + 2];
#pragma unroll
        for (int d = 0; d < DIM; ++d) {
            const double a0 = src[((int64_t)c0 * Lt + k) * DIM + d];
            const double a1 = src[((int64_t)c1 * Lt + k) * DIM + d];
            const double a2 = src[((int64_t)c2 * Lt + k) * DIM + d];
            double o = b.x * a0 + b.y * a1 + b.z * a2;
            if (clamp_neg && o < 0.0) o = 0.0;
            out[d] = o;
        }
    }
    // (vrow: internal vertex -> the caller's row, mops_cell_to_vertex_attr)
    const int64_t o = vrow ? (int64_t)vrow[vid] * Lt + k : idx;
#pragma unroll
    for (int d = 0; d < DIM; ++d) dst[o * DIM + d] = out[d];
}

// ===========================================================================
// seed location: exact 1-NN through a uniform 3-D bucket grid
// ===========================================================================
__device__ __forceinline__ uint64_t bkey(int64_t ix, int64_t iy, int64_t iz) {
    return ((uint64_t)ix << 42) | ((uint64_t)iy << 21) | (uint64_t)iz;
}

__global__ void bucket_keys_kernel(int64_t C, const double4* cxyz, double origin, double h, uint64_t* keys,
                                   int* ids) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C) return;
    const double4 p = cxyz[i];
    const int64_t ix = (int64_t)floor((p.x - origin) / h), iy = (int64_t)floor((p.y - origin) / h),
                  iz = (int64_t)floor((p.z - origin) / h);
    keys[i] = bkey(ix, iy, iz);
    ids[i] = (int)i;
}

// The seed-location bucket index: cells sorted by bucket key, plus a hash
// directory from each non-empty bucket's key to its run of entries, so a
// bucket costs one or two independent probes instead of an 18-step binary
// search (27 per point in the first shell).
struct BucketDir {
    const uint64_t* keys;   // sorted bucket key per entry [C]
    const int* ids;         // cell id per entry [C]
    const uint64_t* hkeys;  // [hmask + 1] bucket key, or kEmptyKey
    const int2* hval;       // {first entry, entry count}
    uint32_t hmask;
};
constexpr uint64_t kEmptyKey = ~0ULL;  // bucket keys use 63 bits

__device__ __forceinline__ uint32_t dir_hash(uint64_t k) {  // splitmix64 finaliser
    k ^= k >> 30; k *= 0xbf58476d1ce4e5b9ULL;
    k ^= k >> 27; k *= 0x94d049bb133111ebULL;
    k ^= k >> 31;
    return (uint32_t)k;
}

__device__ __forceinline__ int2 dir_find(const BucketDir& bd, uint64_t key) {
    uint32_t slot = dir_hash(key) & bd.hmask;
    for (;;) {  // terminates: the table is at most half full
        const uint64_t k = bd.hkeys[slot];
        if (k == key) return bd.hval[slot];
        if (k == kEmptyKey) return make_int2(0, 0);
        slot = (slot + 1) & bd.hmask;
    }
}

// one thread per sorted entry; the first entry of each bucket's run inserts it
__global__ void bucket_dir_kernel(int64_t C, const uint64_t* keys, uint64_t* hkeys, int2* hval, uint32_t hmask) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C) return;
    const uint64_t key = keys[i];
    if (i > 0 && keys[i - 1] == key) return;
    int64_t j = i + 1;
    while (j < C && keys[j] == key) ++j;
    uint32_t slot = dir_hash(key) & hmask;
    for (;;) {
        const unsigned long long prev =
            atomicCAS(reinterpret_cast<unsigned long long*>(hkeys + slot), (unsigned long long)kEmptyKey,
                      (unsigned long long)key);
        if (prev == (unsigned long long)kEmptyKey) {
            hval[slot] = make_int2((int)i, (int)(j - i));
            return;
        }
        slot = (slot + 1) & hmask;
    }
}

__device__ __forceinline__ void consider(const double4* cxyz, int cid, double qx, double qy, double qz, double& best,
                                         int& bi, int exclude, const int* excl = nullptr, int n_excl = 0) {
    if (cid == exclude) return;
    for (int k = 0; k < n_excl; ++k)
        if (cid == excl[k]) return;
    const double4 p = cxyz[cid];
    const double d0 = qx - p.x, d1 = qy - p.y, d2 = qz - p.z;
    double dd = 0.0;
    dd += d0 * d0; dd += d1 * d1; dd += d2 * d2;
    if (dd < best || (dd == best && cid < bi)) { best = dd; bi = cid; }
}

// Exact nearest cell centre to q (smallest id on ties), `exclude` skipped: bucket shells
// around q until the best distance is provably final, else an exhaustive scan.
__device__ int nearest_centre(double qx, double qy, double qz, int64_t C, const double4* cxyz, const BucketDir& bd,
                              double origin, double h, int exclude, double& best,
                              const int* excl = nullptr, int n_excl = 0) {
    best = INFINITY;
    int bi = -1;
    const int kMaxShell = 6;
    const int64_t kLim = (int64_t)1 << 21;
    bool done = false;
    if (isfinite(qx) && isfinite(qy) && isfinite(qz)) {
        const int64_t bx = (int64_t)floor((qx - origin) / h), by = (int64_t)floor((qy - origin) / h),
                      bz = (int64_t)floor((qz - origin) / h);
        for (int s = 0; s <= kMaxShell && !done; ++s) {
            for (int dx = -s; dx <= s; ++dx)
                for (int dy = -s; dy <= s; ++dy)
                    for (int dz = -s; dz <= s; ++dz) {
                        const int m = max(abs(dx), max(abs(dy), abs(dz)));
                        if (m != s) continue;
                        const int64_t ix = bx + dx, iy = by + dy, iz = bz + dz;
                        if (ix < 0 || iy < 0 || iz < 0 || ix >= kLim || iy >= kLim || iz >= kLim) continue;
                        const int2 run = dir_find(bd, bkey(ix, iy, iz));
                        for (int j = run.x; j < run.x + run.y; ++j)
                            consider(cxyz, bd.ids[j], qx, qy, qz, best, bi, exclude, excl, n_excl);
                    }
            // every point outside shells 0..s is at least s*h away
            const double bound = (double)s * h;
            if (bi >= 0 && best <= bound * bound) done = true;
        }
        if (!done) {  // far from every cell centre: exhaustive scan
            for (int64_t cid = 0; cid < C; ++cid) consider(cxyz, (int)cid, qx, qy, qz, best, bi, exclude, excl, n_excl);
        }
    }
    return bi;
}

// MPASOField::calcInWhichCells (MPASOField.cpp:23-34): exact 1-NN over the cell centres.
// With `hint` (a candidate cell per point, e.g. the cell a chained particle ended the
// previous pair in): if q lies within rloc(h) = d_nn(h)/2 - 1 m of centre h, where d_nn(h)
// is the distance from h to the nearest OTHER centre, then every other centre c' has
// |q - c'| >= d_nn - |q - h| > |q - h| + 2 m, so h is the unique exact answer and the
// search is skipped.  Any hint (or none) gives the same result.
//
// A point outside that ball (near an edge of the hint's cell) is resolved among the hint
// and its cellsOnCell neighbours S when that is provably exact: every centre outside S is
// at least ring(h) = the distance from h's centre to the nearest centre not in S away from
// h's centre, hence at least ring(h) - |q - h| from q; if that exceeds the best distance
// within S by a 1 m margin, the best of S (same tie rule) is the global answer.
__global__ void locate_kernel(int64_t n, const double* pts, int64_t C, const double4* cxyz, BucketDir bd,
                              double origin, double h, int origin_cell, const int* hint,
                              const double* rloc2, const double* ring, const int* cellrec, int rec_ints,
                              int maxv, int* out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double qx = pts[3 * i], qy = pts[3 * i + 1], qz = pts[3 * i + 2];
    // (0,0,0) is where a particle that died before its first record continues
    // from in a pair chain (lastPoint = 0, quirk Q1); its exact answer is
    // precomputed instead of scanning every cell
    if (qx == 0.0 && qy == 0.0 && qz == 0.0) { out[i] = origin_cell; return; }
    if (hint) {
        const int hc = hint[i];
        if (hc >= 0 && hc < C) {
            const double4 p = cxyz[hc];
            const double d0 = qx - p.x, d1 = qy - p.y, d2 = qz - p.z;
            const double dh2 = d0 * d0 + d1 * d1 + d2 * d2;
            if (dh2 < rloc2[hc]) { out[i] = hc; return; }
            double best = INFINITY;
            int bi = -1;
            consider(cxyz, hc, qx, qy, qz, best, bi, -1);
            const int* r = cellrec + (int64_t)hc * rec_ints;
            const int nv = r[0];
            for (int k = 0; k < nv && k < maxv; ++k) {
                const int nb = r[1 + maxv + k];
                if (nb >= 0) consider(cxyz, nb, qx, qy, qz, best, bi, -1);
            }
            if (bi >= 0 && isfinite(dh2) && ring[hc] - sqrt(dh2) > sqrt(best) * (1.0 + 1e-9) + 1.0) {
                out[i] = bi;
                return;
            }
        }
    }
    double best;
    out[i] = nearest_centre(qx, qy, qz, C, cxyz, bd, origin, h, -1, best);
}

// rloc(c)^2 for the hinted locate: half the distance to the nearest other centre, shrunk
// by 1e-9 relative and 1 m absolute (>> the rounding of |q - c| at Earth radius); -1 when
// another centre coincides with c (never taken)
__global__ void locate_radius_kernel(int64_t C, const double4* cxyz, BucketDir bd,
                                     double origin, double h, const int* cellrec, int rec_ints, int maxv,
                                     double* rloc2, double* ring) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const double4 p = cxyz[c];
    // ring(c): distance to the nearest centre outside {c} + cellsOnCell[c] (the hinted
    // locate's local set), shrunk by 1e-9 relative and 1 m; -inf if there is none
    {
        const int* r = cellrec + c * rec_ints;
        const int nv = min(r[0], maxv);
        double b2;
        const int o = nearest_centre(p.x, p.y, p.z, C, cxyz, bd, origin, h, (int)c, b2, r + 1 + maxv, nv);
        ring[c] = (o >= 0 && isfinite(b2)) ? sqrt(b2) * (1.0 - 1e-9) - 1.0 : -INFINITY;
    }
    double best;
    const int nb = nearest_centre(p.x, p.y, p.z, C, cxyz, bd, origin, h, (int)c, best);
    double r2 = -1.0;
    if (nb < 0) {
        r2 = INFINITY;  // the only centre: every point's nearest
    } else if (best > 0.0 && isfinite(best)) {
        const double r = 0.5 * sqrt(best) * (1.0 - 1e-9) - 1.0;
        if (r > 0.0) r2 = r * r * (1.0 - 1e-9);
    }
    rloc2[c] = r2;
}

// ===========================================================================
// fast-path flags and particle locality order
// ===========================================================================

// Fast-path word per cell (see dev::fast_ok).  Two passes: per-vertex facts
// from one coalesced (vertex, level) element per thread -- vfail: the first
// level l that is non-finite, has |z| > 1e6 m or (l > 0) does not drop below
// z_{l-1} - 1e-6 m (every level's test reads the raw z_{l-1}, exactly as a
// per-column scan would; L if none); vzero: every level is 0 -- then a
// per-cell pass over the polygon's vertices.
__global__ void fill_i32_kernel(int64_t n, int32_t v, int32_t* __restrict__ p) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = v;
}

__global__ void vertex_mono_kernel(int64_t V, int L, const double* __restrict__ zt, int32_t* __restrict__ vfail,
                                   uint8_t* __restrict__ vzero) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= V * L) return;
    const int l = (int)(i % L);
    const double z = zt[i];
    bool ok = isfinite(z) && fabs(z) <= 1e6;
    if (l > 0) ok = ok && (z < zt[i - 1] - 1e-6);
    if (!ok) {
        // only the first level of each failing run competes for the minimum
        bool prev_ok = true;
        if (l > 0) {
            const double zp = zt[i - 1];
            prev_ok = isfinite(zp) && fabs(zp) <= 1e6;
            if (l > 1) prev_ok = prev_ok && (zp < zt[i - 2] - 1e-6);
        }
        if (l == 0 || prev_ok) atomicMin(&vfail[i / L], l);
    }
    if (z != 0.0) vzero[i / L] = 0;  // every writer stores 0: the race is benign
}

__global__ void mono_kernel(int64_t C, int maxv, int rec_ints, const int* cellrec, const int32_t* vfail,
                            const uint8_t* vzero, int L, uint32_t* mono) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C) return;
    const int* r = cellrec + i * rec_ints;
    const int nv = r[0];
    bool ok = (nv >= 1 && nv <= kMaxVertex && L >= 2);
    bool any_dec = false;
    int km = L - 1;
    uint32_t zmask = 0u;
    for (int k = 0; k < nv && ok; ++k) {
        const int v = r[1 + k];
        if (vzero[v]) {
            zmask |= 1u << k;
        } else {
            any_dec = true;
            km = min(km, vfail[v] - 1);  // levels 0..vfail-1 are good
        }
    }
    ok = ok && any_dec && km >= 1;
    mono[i] = ok ? (0x80000000u | ((uint32_t)km << 20) | zmask) : 0u;
}

// The neighbour table of dev::nbr_stay (maxEdges <= 7): the centre c (doubles), the offsets q_k - c of
// cellsOnCell slot k rounded to float (zero when not considered), and the mask of the slots the walk
// considers (dev::walk's ok[k]: k < nEdges, a valid id).
__global__ void cell_nbr_kernel(int64_t C, const int* __restrict__ cellrec, const double4* __restrict__ cxyz,
                                uint4* __restrict__ nbr) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    constexpr int MAXV = 7, REC = ((1 + 2 * MAXV) + 3) / 4 * 4;
    const int* r = cellrec + c * REC;
    const int nv = r[0];
    const double4 q = cxyz[c];
    uint32_t w[4 * kNbrQ];
    w[0] = (uint32_t)__double2loint(q.x); w[1] = (uint32_t)__double2hiint(q.x);
    w[2] = (uint32_t)__double2loint(q.y); w[3] = (uint32_t)__double2hiint(q.y);
    w[4] = (uint32_t)__double2loint(q.z); w[5] = (uint32_t)__double2hiint(q.z);
    uint32_t mask = 0;
    for (int k = 0; k < MAXV; ++k) {
        const int id = r[1 + MAXV + k];
        const bool ok = k < nv && id >= 0 && id < C;
        float d[3] = {0.0f, 0.0f, 0.0f};
        if (ok) {
            const double4 n = cxyz[id];
            d[0] = (float)(n.x - q.x); d[1] = (float)(n.y - q.y); d[2] = (float)(n.z - q.z);
            mask |= 1u << k;
        }
        for (int j = 0; j < 3; ++j) w[6 + 3 * k + j] = __float_as_uint(d[j]);
    }
    w[27] = mask;
    for (int j = 0; j < kNbrQ; ++j) nbr[c * kNbrQ + j] = make_uint4(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]);
}

// d_cpoly's 16-B pieces by cell rank: piece p (slot p / 2, half p % 2) of the cell of rank r at p * C + r
__global__ void cpoly_rank_kernel(int64_t C, const int* __restrict__ rank_cell, const double4* __restrict__ cpoly,
                                  double2* __restrict__ cpolyr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C * 14) return;
    const int64_t p = i / C, r = i - p * C;
    cpolyr[i] = reinterpret_cast<const double2*>(cpoly)[(int64_t)rank_cell[r] * 14 + p];
}

// Each cell's polygon in the evaluation's rotated slot order (dev::Cell: slot j holds
// poly[j-1], slot 0 poly[nv-1]) packed with its Wachspress numerator B_j = area(poly[j-1],
// poly[j], poly[j+1]) -- the same device arithmetic as the in-kernel computation, so
// bit-identical -- as one 32-B {x, y, z, B_j} per slot: the modes that re-read the polygon per
// evaluation (pathline) load a slot with 2 VMEM instructions instead of a vertex double4 + B_j.
// ... and (cnrm != NULL, MAXV 7) the IsInMesh edge normals n_i = X_i x X_{i+1} of the rotated slots,
// the products load_cell and dev::weights form (same operands, same order), [C][kCellNrm]: the
// cooperative waves' tile takes them from here
template <int MAXV>
__global__ void cell_poly_kernel(int64_t C, const int* cellrec, const double4* vxyz, double4* cpoly,
                                 double* cnrm = nullptr, double* cedge = nullptr) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    constexpr int REC = ((1 + 2 * MAXV) + 3) / 4 * 4;
    const int* r = cellrec + c * REC;
    const int nv = r[0];
    double x[MAXV], y[MAXV], z[MAXV];
#pragma unroll
    for (int k = 0; k < MAXV; ++k) {
        if (k < nv) { const double4 p = vxyz[r[1 + k]]; x[k] = p.x; y[k] = p.y; z[k] = p.z; }
        else { x[k] = 0.0; y[k] = 0.0; z[k] = 0.0; }
    }
    double lx = 0, ly = 0, lz = 0;
#pragma unroll
    for (int k = 0; k < MAXV; ++k)
        if (k == nv - 1) { lx = x[k]; ly = y[k]; lz = z[k]; }
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
        double4 o = make_double4(0.0, 0.0, 0.0, 0.0);
        if (i < nv) {
            const double qx = (i == 0) ? lx : x[(i + MAXV - 1) % MAXV];
            const double qy = (i == 0) ? ly : y[(i + MAXV - 1) % MAXV];
            const double qz = (i == 0) ? lz : z[(i + MAXV - 1) % MAXV];
            const bool wrap = (i + 1 >= nv);
            const double nx = wrap ? x[0] : x[(i + 1) % MAXV];
            const double ny = wrap ? y[0] : y[(i + 1) % MAXV];
            const double nz = wrap ? z[0] : z[(i + 1) % MAXV];
            o = make_double4(qx, qy, qz, dev::wach_numerator(dev::tri_area(qx, qy, qz, x[i], y[i], z[i], nx, ny, nz)));
        }
        cpoly[c * MAXV + i] = o;
        if (cedge && 3 * i + 2 < kCellNrm) {  // b - a of the weights' tri_area for slot i (X_{i+1} = poly[i])
            double* e = cedge + c * kCellNrm + 3 * i;
            e[0] = i < nv ? x[i] - o.x : 0.0;
            e[1] = i < nv ? y[i] - o.y : 0.0;
            e[2] = i < nv ? z[i] - o.z : 0.0;
        }
        if (cnrm && 3 * i + 2 < kCellNrm) {
            double* n = cnrm + c * kCellNrm + 3 * i;
            if (i < nv) {  // X_i = (qx, qy, qz), X_{i+1} = poly[i] = (x[i], y[i], z[i])
                n[0] = o.y * z[i] - o.z * y[i];
                n[1] = o.z * x[i] - o.x * z[i];
                n[2] = o.x * y[i] - o.y * x[i];
            } else {
                n[0] = 0.0; n[1] = 0.0; n[2] = 0.0;
            }
        }
    }
    if (cnrm) cnrm[c * kCellNrm + kCellNrm - 1] = 0.0;
    if (cedge) cedge[c * kCellNrm + kCellNrm - 1] = 0.0;
}

// Level-pair records (mops_field::d_pr), one 16-B chunk per thread so that a wave's
// stores are contiguous: chunk q of record (v, k) is {z_{k-1}, z_k}, {w_{k-1}, w_k} or
// two of the six doubles vel_{k-1}.xyz, vel_k.xyz.  IDX = uint32_t when the chunk count fits.
template <typename IDX>
__global__ void pair_record_kernel(int64_t V, int L, const double* __restrict__ zt, const double* __restrict__ vel,
                                   const double* __restrict__ w, double* __restrict__ pr) {
    const IDX j = (IDX)blockIdx.x * (IDX)blockDim.x + (IDX)threadIdx.x;
    if ((int64_t)j >= V * (L - 1) * (kPairRec / 2)) return;
    // (k-1, q, v) with v fastest (piece-major: contiguous stores), or (k-1, v, q) record-major
    const IDX vv = (IDX)V;
    IDX v;
    int q, k;
    if (MOPS_PR_PIECES) {
        const IDX r = j / vv;
        v = j - r * vv;
        q = (int)(r % (IDX)(kPairRec / 2));
        k = (int)(r / (IDX)(kPairRec / 2)) + 1;
    } else {
        const IDX rec = j / (IDX)(kPairRec / 2);
        q = (int)(j - rec * (IDX)(kPairRec / 2));
        const IDX kk = rec / vv;
        v = rec - kk * vv;
        k = (int)kk + 1;
    }
    double2 val;
    if (q == 0) {
        const double* z = zt + (int64_t)v * L;
        val = make_double2(z[k - 1], z[k]);
    } else if (q == 1) {
        const double* ww = w + (int64_t)v * (L + 1);
        val = make_double2(ww[k - 1], ww[k]);
    } else {
        const double* u = vel + ((int64_t)v * L + k - 1) * 3 + 2 * (q - 2);
        val = make_double2(u[0], u[1]);
    }
    reinterpret_cast<double2*>(pr)[pr_base((uint32_t)(k - 1), (uint32_t)v, (uint32_t)V) +
                                   (uint32_t)q * pr_qstride((uint32_t)V)] = val;
}

// Level-major records ((k-1)*V + v) from the vertex-major zt/vel/w arrays: a block stages a
// tile of kRecTV vertices x (kRecTK + 1) levels through LDS (reads run along each vertex's
// column) and writes kRecTK rows of kRecTV consecutive records (contiguous 5 KB per row), so
// both sides are coalesced.  Same values and chunk layout as pair_record_kernel.
#ifndef MOPS_REC_TV
#define MOPS_REC_TV 32  // 32 x 16 tiles: 16.4 vs 17.6 ms per oRRS18to6 snapshot (64 x 16), profiles/r03
#endif
#ifndef MOPS_REC_TK
#define MOPS_REC_TK 16
#endif
constexpr int kRecTV = MOPS_REC_TV, kRecTK = MOPS_REC_TK;
#ifndef MOPS_REC_TILED
#define MOPS_REC_TILED 1  // records built by pair_record_tiled_kernel (0: one 16-B piece per thread, pair_record_kernel)
#endif
__global__ void __launch_bounds__(256) pair_record_tiled_kernel(int64_t V, int L, const double* __restrict__ zt,
                                                                const double* __restrict__ vel,
                                                                const double* __restrict__ w,
                                                                double* __restrict__ pr) {
    __shared__ double sz[kRecTV][kRecTK + 1], sw[kRecTV][kRecTK + 1], su[kRecTV][kRecTK + 1][3];
    const int64_t v0 = (int64_t)blockIdx.x * kRecTV;
    const int k0 = (int)blockIdx.y * kRecTK;  // rows k-1 = k0 .. k0+nk-1 use levels k0 .. k0+nk
    const int nk = min(kRecTK, L - 1 - k0);
    const int nv = (int)min<int64_t>(kRecTV, V - v0);
    const int t = (int)threadIdx.x;
    for (int i = t; i < kRecTV * (kRecTK + 1); i += blockDim.x) {
        const int vl = i / (kRecTK + 1), kl = i - vl * (kRecTK + 1);
        if (vl < nv && kl <= nk) {
            const int64_t v = v0 + vl;
            sz[vl][kl] = zt[v * L + k0 + kl];
            sw[vl][kl] = w[v * (L + 1) + k0 + kl];
        }
    }
    for (int i = t; i < kRecTV * (kRecTK + 1) * 3; i += blockDim.x) {
        const int vl = i / ((kRecTK + 1) * 3), r = i - vl * ((kRecTK + 1) * 3), kl = r / 3;
        if (vl < nv && kl <= nk) su[vl][kl][r - kl * 3] = vel[((v0 + vl) * L + k0) * 3 + r];
    }
    __syncthreads();
    for (int i = t; i < nk * kRecTV * (kPairRec / 2); i += blockDim.x) {
        // piece-major: consecutive threads on consecutive vertices of one (level, piece) row
        int q, kl, vl;
        if (MOPS_PR_PIECES) {
            vl = i % kRecTV;
            const int r = i / kRecTV;
            q = r % (kPairRec / 2); kl = r / (kPairRec / 2);
        } else {
            const int rl = i / (kPairRec / 2);
            q = i - rl * (kPairRec / 2); kl = rl / kRecTV; vl = rl - kl * kRecTV;
        }
        if (vl >= nv) continue;
        double2 val;
        if (q == 0) val = make_double2(sz[vl][kl], sz[vl][kl + 1]);
        else if (q == 1) val = make_double2(sw[vl][kl], sw[vl][kl + 1]);
        else if (q == 2) val = make_double2(su[vl][kl][0], su[vl][kl][1]);
        else if (q == 3) val = make_double2(su[vl][kl][2], su[vl][kl + 1][0]);
        else val = make_double2(su[vl][kl + 1][1], su[vl][kl + 1][2]);
        reinterpret_cast<double2*>(pr)[pr_base((uint32_t)(k0 + kl), (uint32_t)(v0 + vl), (uint32_t)V) +
                                       (uint32_t)q * pr_qstride((uint32_t)V)] = val;
    }
}

// The same level-major records straight from the CELL arrays: each tile's vertex values are the
// barycentric combinations cell_to_vertex_bary_kernel computes (b.x*a0 + b.y*a1 + b.z*a2 of the
// three cellsOnVertex, 0 at a boundary vertex; same operands, same order: the same doubles), so the
// vertex velocity and vertical-velocity arrays are never written and read back (36 GB of traffic
// per oRRS18to6 snapshot).  Also writes the vertex zTop (the bracket's column) and w at level L,
// the one value no record holds.
template <bool HAS_W>
__global__ void __launch_bounds__(256) pair_record_fused_kernel(int64_t V, int L, const int* __restrict__ cov,
                                                                const double4* __restrict__ bary,
                                                                const double* __restrict__ ztc,
                                                                const double* __restrict__ velc,
                                                                const double* __restrict__ wc,
                                                                double* __restrict__ zt, double* __restrict__ w_out,
                                                                double* __restrict__ pr) {
    __shared__ double sz[kRecTV][kRecTK + 1], sw[kRecTV][kRecTK + 1], su[kRecTV][kRecTK + 1][3];
    const int64_t v0 = (int64_t)blockIdx.x * kRecTV;
    const int k0 = (int)blockIdx.y * kRecTK;
    const int nk = min(kRecTK, L - 1 - k0);
    const int nv = (int)min<int64_t>(kRecTV, V - v0);
    const int t = (int)threadIdx.x;
    const bool last = k0 + nk == L - 1;  // this tile row holds level L-1
    for (int i = t; i < kRecTV * (kRecTK + 1); i += blockDim.x) {
        const int vl = i / (kRecTK + 1), kl = i - vl * (kRecTK + 1);
        if (vl < nv && kl <= nk) {
            const int64_t v = v0 + vl;
            const int k = k0 + kl;
            const double4 b = bary[v];
            double z = 0.0, w = 0.0, u0 = 0.0, u1 = 0.0, u2 = 0.0, wl = 0.0;
            if (b.w != 0.0) {
                const int64_t c0 = cov[3 * v], c1 = cov[3 * v + 1], c2 = cov[3 * v + 2];
                z = b.x * ztc[c0 * L + k] + b.y * ztc[c1 * L + k] + b.z * ztc[c2 * L + k];
                const double* a0 = velc + (c0 * L + k) * 3;
                const double* a1 = velc + (c1 * L + k) * 3;
                const double* a2 = velc + (c2 * L + k) * 3;
                u0 = b.x * a0[0] + b.y * a1[0] + b.z * a2[0];
                u1 = b.x * a0[1] + b.y * a1[1] + b.z * a2[1];
                u2 = b.x * a0[2] + b.y * a1[2] + b.z * a2[2];
                if constexpr (HAS_W) {
                    w = b.x * wc[c0 * (L + 1) + k] + b.y * wc[c1 * (L + 1) + k] + b.z * wc[c2 * (L + 1) + k];
                    if (last && kl == nk)
                        wl = b.x * wc[c0 * (L + 1) + L] + b.y * wc[c1 * (L + 1) + L] + b.z * wc[c2 * (L + 1) + L];
                }
            }
            sz[vl][kl] = z; sw[vl][kl] = w;
            su[vl][kl][0] = u0; su[vl][kl][1] = u1; su[vl][kl][2] = u2;
            if (kl < nk || last) zt[v * L + k] = z;  // (levels shared by two tile rows written once)
            if (last && kl == nk) w_out[v * (L + 1) + L] = wl;
        }
    }
    __syncthreads();
    for (int i = t; i < nk * kRecTV * (kPairRec / 2); i += blockDim.x) {
        // piece-major: consecutive threads on consecutive vertices of one (level, piece) row
        int q, kl, vl;
        if (MOPS_PR_PIECES) {
            vl = i % kRecTV;
            const int r = i / kRecTV;
            q = r % (kPairRec / 2); kl = r / (kPairRec / 2);
        } else {
            const int rl = i / (kPairRec / 2);
            q = i - rl * (kPairRec / 2); kl = rl / kRecTV; vl = rl - kl * kRecTV;
        }
        if (vl >= nv) continue;
        double2 val;
        if (q == 0) val = make_double2(sz[vl][kl], sz[vl][kl + 1]);
        else if (q == 1) val = make_double2(sw[vl][kl], sw[vl][kl + 1]);
        else if (q == 2) val = make_double2(su[vl][kl][0], su[vl][kl][1]);
        else if (q == 3) val = make_double2(su[vl][kl][2], su[vl][kl + 1][0]);
        else val = make_double2(su[vl][kl + 1][1], su[vl][kl + 1][2]);
        reinterpret_cast<double2*>(pr)[pr_base((uint32_t)(k0 + kl), (uint32_t)(v0 + vl), (uint32_t)V) +
                                       (uint32_t)q * pr_qstride((uint32_t)V)] = val;
    }
}

// mops_field_export of a fused field: the vertex velocity [V][L][3] and vertical velocity levels
// 0..L-1 back out of the level-major records (level j from record j, level L-1 from record L-2)
__global__ void records_to_vertex_kernel(int64_t V, int L, const double* __restrict__ pr, double* __restrict__ vel,
                                         double* __restrict__ w) {
    const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (idx >= V * L) return;
    const int64_t v = idx / L;
    const int j = (int)(idx - v * L);
    const bool hi = j == L - 1;  // the second half of record L-2
    const double2* p2 = reinterpret_cast<const double2*>(pr);
    const uint32_t b = pr_base((uint32_t)(hi ? j - 1 : j), (uint32_t)v, (uint32_t)V), qs = pr_qstride((uint32_t)V);
    double r[kPairRec];  // the record's 10 doubles in their order
#pragma unroll
    for (int q = 0; q < kPairRec / 2; ++q) {
        const double2 x = p2[b + (uint32_t)q * qs];
        r[2 * q] = x.x; r[2 * q + 1] = x.y;
    }
    w[v * (L + 1) + j] = hi ? r[3] : r[2];
    vel[idx * 3 + 0] = hi ? r[7] : r[4];
    vel[idx * 3 + 1] = hi ? r[8] : r[5];
    vel[idx * 3 + 2] = hi ? r[9] : r[6];
}

__device__ __forceinline__ uint64_t spread3(uint64_t v) {  // 21 bits -> every third bit
    v &= 0x1fffffULL;
    v = (v | (v << 32)) & 0x1f00000000ffffULL;
    v = (v | (v << 16)) & 0x1f0000ff0000ffULL;
    v = (v | (v << 8)) & 0x100f00f00f00f00fULL;
    v = (v | (v << 4)) & 0x10c30c30c30c30c3ULL;
    v = (v | (v << 2)) & 0x1249249249249249ULL;
    return v;
}

__global__ void cell_key_kernel(int64_t C, const double4* cxyz, uint64_t* key, int* ids) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= C) return;
    ids[i] = (int)i;
    const double4 p = cxyz[i];
    const double r = sqrt(p.x * p.x + p.y * p.y + p.z * p.z);
    const double s = (r > 0.0) ? 1.0 / r : 0.0;
    const double m = 2097151.0;
    const uint64_t qx = (uint64_t)fmin(fmax((p.x * s * 0.5 + 0.5) * m, 0.0), m);
    const uint64_t qy = (uint64_t)fmin(fmax((p.y * s * 0.5 + 0.5) * m, 0.0), m);
    const uint64_t qz = (uint64_t)fmin(fmax((p.z * s * 0.5 + 0.5) * m, 0.0), m);
    key[i] = (spread3(qx) << 2) | (spread3(qy) << 1) | spread3(qz);
}

// rank[c] = position of cell c in the Morton order of the cell centres (ties by cell id)
__global__ void cell_rank_kernel(int64_t C, const int* sorted_ids, uint32_t* rank) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < C) rank[sorted_ids[i]] = (uint32_t)i;
}

// Sort bits of a particle key: ranks are < C and the "last" key is C itself
inline int particle_key_bits(int64_t C) {
    int b = 1;
    while (b < 31 && ((int64_t)1 << b) <= C) ++b;
    return b;
}

// Morton rank of each particle's cell; a dead particle (death >= 0, when given) or one without a
// cell sorts last (key C), so live particles fill whole waves and all-dead waves exit at once.
// 32-bit keys over particle_key_bits(C) bits: 3 radix passes at C ~ 2.4e5 instead of 8 over a
// 64-bit Morton key.
__global__ void particle_key_kernel(int64_t n, int64_t C, const int* cell, const int* death,
                                    const uint32_t* cell_rank, uint32_t* key, int* idx, int* n_live) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    bool sorts_first = false;
    if (i < n) {
        const int c = cell[i];
        const bool live = !death || death[i] < 0;
        sorts_first = live && c >= 0 && c < C;
        key[i] = sorts_first ? cell_rank[c] : (uint32_t)C;
        idx[i] = (int)i;
    }
    if (n_live) {  // one atomic per wave: the particles that sort before the ~0 keys
        const unsigned long long m = __ballot(sorts_first);
        if (__lane_id() == 0 && m) atomicAdd(n_live, (int)__popcll(m));
    }
}

// Gather of up to kPermMax SoA arrays (and record rows) by a slot order in one launch:
// dst[row][i] = src[row][order[i]] (order NULL = copy); blockIdx.y enumerates (array, row).
constexpr int kPermMax = 16;
struct PermArrays {
    const char* src[kPermMax];
    char* dst[kPermMax];
    int64_t stride_bytes[kPermMax];  // bytes between consecutive rows
    int elem[kPermMax];              // bytes per element: 4, 8 or 24
    int row0[kPermMax + 1];          // first blockIdx.y row of each array (prefix over rows)
    int count;
};
__global__ void permute_kernel(int64_t n, const int32_t* __restrict__ order, PermArrays a) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int y = blockIdx.y;
    int k = 0;
    while (k + 1 < a.count && a.row0[k + 1] <= y) ++k;  // the array this row belongs to (uniform)
    const int64_t r = y - a.row0[k];
    const int64_t j = order ? (int64_t)order[i] : i;
    const char* src = a.src[k] + r * a.stride_bytes[k];
    char* dst = a.dst[k] + r * a.stride_bytes[k];
    switch (a.elem[k]) {
        case 4: reinterpret_cast<int32_t*>(dst)[i] = reinterpret_cast<const int32_t*>(src)[j]; break;
        case 8: reinterpret_cast<double*>(dst)[i] = reinterpret_cast<const double*>(src)[j]; break;
        default: {
            const double* q = reinterpret_cast<const double*>(src) + 3 * j;
            double* o = reinterpret_cast<double*>(dst) + 3 * i;
            o[0] = q[0]; o[1] = q[1]; o[2] = q[2];
        }
    }
}

// ===========================================================================
// host side
// ===========================================================================
namespace {

template <typename T>
mops_status dmalloc(T** p, size_t count, int64_t* acc) {
    if (count == 0) count = 1;
    hipError_t e = hipMalloc(reinterpret_cast<void**>(p), count * sizeof(T));
    if (e != hipSuccess) return fail(MOPS_ERR_HIP, std::string("hipMalloc failed: ") + hipGetErrorString(e));
    if (acc) *acc += (int64_t)(count * sizeof(T));
    return MOPS_OK;
}

#define MOPS_TRY(expr)                 \
    do {                               \
        mops_status _s = (expr);       \
        if (_s != MOPS_OK) return _s;  \
    } while (0)

inline unsigned grid_for(int64_t n) { return (unsigned)((n + kBlock - 1) / kBlock); }

// 63-bit Morton key of a vertex direction (the cell_key_kernel quantisation, on the host)
uint64_t vertex_morton_key(double x, double y, double z) {
    auto spread = [](uint64_t v) {
        v &= 0x1fffffULL;
        v = (v | (v << 32)) & 0x1f00000000ffffULL;
        v = (v | (v << 16)) & 0x1f0000ff0000ffULL;
        v = (v | (v << 8)) & 0x100f00f00f00f00fULL;
        v = (v | (v << 4)) & 0x10c30c30c30c30c3ULL;
        v = (v | (v << 2)) & 0x1249249249249249ULL;
        return v;
    };
    const double r = std::sqrt(x * x + y * y + z * z);
    const double sc = (r > 0.0 && std::isfinite(r)) ? 1.0 / r : 0.0;
    const double m = 2097151.0;
    auto q = [&](double a) { return (uint64_t)std::fmin(std::fmax((a * sc * 0.5 + 0.5) * m, 0.0), m); };
    return (spread(q(x)) << 2) | (spread(q(y)) << 1) | spread(q(z));
}

int pick_maxv(int maxE) {
    if (maxE <= 7) return 7;
    if (maxE <= 12) return 12;
    return 20;
}

mops_status upload_xyz(const double* h, int64_t n, double4** d, int64_t* acc, hipStream_t s) {
    std::vector<double4> tmp((size_t)n);
    for (int64_t i = 0; i < n; ++i) tmp[i] = make_double4(h[3 * i], h[3 * i + 1], h[3 * i + 2], 0.0);
    MOPS_TRY(dmalloc(d, (size_t)n, acc));
    HIP_TRY(hipMemcpyAsync(*d, tmp.data(), n * sizeof(double4), hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
    return MOPS_OK;
}

template <typename T>
mops_status upload(const T* h, size_t count, T** d, int64_t* acc, hipStream_t s) {
    MOPS_TRY(dmalloc(d, count, acc));
    HIP_TRY(hipMemcpyAsync(*d, h, count * sizeof(T), hipMemcpyHostToDevice, s));
    return MOPS_OK;
}

void free_mesh(mops_mesh* m) {
    if (!m) return;
    (void)hipFree(m->d_cellrec); (void)hipFree(m->d_cxyz); (void)hipFree(m->d_vxyz); (void)hipFree(m->d_cov);
    (void)hipFree(m->d_bary);
    (void)hipFree(m->d_bkeys); (void)hipFree(m->d_bcells); (void)hipFree(m->d_hkeys); (void)hipFree(m->d_hval); (void)hipFree(m->d_cell_rank); (void)hipFree(m->d_rank_cell); (void)hipFree(m->d_cpolyr); (void)hipFree(m->d_cpoly); (void)hipFree(m->d_cnrm); (void)hipFree(m->d_cedge); (void)hipFree(m->d_nbr); (void)hipFree(m->d_rloc2); (void)hipFree(m->d_ring);
    (void)hipFree(m->d_scratch);
    (void)hipFree(m->d_eoc); (void)hipFree(m->d_coe); (void)hipFree(m->d_exyz); (void)hipFree(m->d_rbf_coef);
    (void)hipFree(m->d_rbf_slot);
    for (auto& f : m->coop_flags) (void)hipFree(f.second);
    (void)hipFree(m->d_vold);
    delete m;
}

void free_field(mops_field* f) {
    if (!f) return;
    (void)hipFree(f->d_zt); (void)hipFree(f->d_vel); (void)hipFree(f->d_w); (void)hipFree(f->d_mono); (void)hipFree(f->d_vmono);
    (void)hipFree(f->d_vzero);
    (void)hipFree(f->d_pr);
    (void)hipFree(f->d_ztc); (void)hipFree(f->d_velc);
    delete f;
}

}  // namespace

BucketDir bucket_dir(const mops_mesh* m) {
    return BucketDir{m->d_bkeys, m->d_bcells, m->d_hkeys, m->d_hval, m->hmask};
}

int64_t gcd64(int64_t a, int64_t b) {
    while (b) { int64_t t = a % b; a = b; b = t; }
    return a;
}

// Which pathline-Euler instantiation runs a launch: the cooperative tile pays where a wave's lanes
// share few cells (configs 3 and 5: 40+ particles per cell), the plain kernel where they do not (config
// 4: ~3 per cell, ~20 cells per wave).  One block samples up to 4096 of the launch's 64-slot waves in
// the current (locality) order, counts the runs of equal cells in each, and writes flag = 1 when the
// mean is at most MOPS_COOP_CELLS -- on the device, so the host never waits.
#ifndef MOPS_COOP_CELLS
#define MOPS_COOP_CELLS 6
#endif
__global__ void __launch_bounds__(256) coop_select_kernel(int64_t n, const int* __restrict__ cell,
                                                          const int* __restrict__ n_live, int* __restrict__ flag) {
    __shared__ unsigned long long runs[256];
    int64_t m = n;
    if (n_live) m = min<int64_t>(m, (int64_t)*n_live);
    const int64_t waves = (m + 63) / 64;
    const int64_t S = waves < 4096 ? waves : 4096;
    unsigned long long r = 0;
    for (int64_t j = threadIdx.x; j < S; j += blockDim.x) {
        const int64_t w = j * waves / S, lo = 64 * w, hi = min<int64_t>(m, lo + 64);
        int prev = cell[lo];
        r += 1;
        for (int64_t i = lo + 1; i < hi; ++i) {
            const int c = cell[i];
            r += (c != prev);
            prev = c;
        }
    }
    runs[threadIdx.x] = r;
    __syncthreads();
    for (int k = blockDim.x / 2; k > 0; k >>= 1) {
        if ((int)threadIdx.x < k) runs[threadIdx.x] += runs[threadIdx.x + k];
        __syncthreads();
    }
    if (threadIdx.x == 0) *flag = (S > 0 && runs[0] <= (unsigned long long)MOPS_COOP_CELLS * (unsigned long long)S) ? 1 : 0;
}

// The stream's instantiation flag (mops_mesh::coop_flags), allocated on the stream's first pathline launch.
static mops_status coop_flag(const mops_mesh* mesh, hipStream_t s, int** out) {
    std::lock_guard<std::mutex> lk(mesh->coop_mu);
    for (const auto& f : mesh->coop_flags)
        if (f.first == s) { *out = f.second; return MOPS_OK; }
    int* d = nullptr;
    HIP_TRY(hipMalloc(reinterpret_cast<void**>(&d), sizeof(int)));
    mesh->coop_flags.emplace_back(s, d);
    *out = d;
    return MOPS_OK;
}

template <int MAXV>
void launch_traj(const TrajArgs& a, bool path, bool euler, hipStream_t s) {
    const unsigned g = (unsigned)((a.n + kTrajBlock - 1) / kTrajBlock);
    if (path) {
        if (euler) {
            if constexpr (MAXV == 7) {  // both instantiations; a.coop_sel lets exactly one of them run
                if (a.coop_sel) traj_kernel<MAXV, true, true, true><<<g, kTrajBlock, 0, s>>>(a);
            }
            traj_kernel<MAXV, true, true><<<g, kTrajBlock, 0, s>>>(a);
        } else {
            if constexpr (MAXV == 7) {
                if (a.coop_sel && a.handoff) traj_kernel<MAXV, true, false, true, true><<<g, kTrajBlock, 0, s>>>(a);
                if (a.coop_sel) traj_kernel<MAXV, true, false, true><<<g, kTrajBlock, 0, s>>>(a);
            }
            traj_kernel<MAXV, true, false><<<g, kTrajBlock, 0, s>>>(a);
        }
    } else {
        if (euler) traj_kernel<MAXV, false, true><<<g, kTrajBlock, 0, s>>>(a);
        else traj_kernel<MAXV, false, false><<<g, kTrajBlock, 0, s>>>(a);
    }
}

// The trajectory kernel's exact fast sqrt / sin / cos / a/|a| restate the device library's and the
// compiler's own expansions (dev::sqrt_core, sincos_small, xdiv_norm3).  A toolchain whose
// expansions changed would break the bit parity silently, so every mesh creation first checks
// them against the library on fixed arguments (the full sweep is mops_selftest_math's test).
static mops_status check_fast_math(hipStream_t s) {
    constexpr int n = 512;  // arguments per op (op 2: n vectors of 3)
    std::vector<double> x(3 * n), out(6 * n);
    double* d = nullptr;  // [3n inputs | 6n outputs]
    HIP_TRY(hipMalloc(&d, 9 * n * sizeof(double)));
    mops_status st = MOPS_OK;
    for (int op = 0; op < 3 && st == MOPS_OK; ++op) {
        const int nin = (op == 2) ? 3 * n : n, width = (op == 0) ? 2 : (op == 1 ? 4 : 2);  // outputs per input
        for (int i = 0; i < nin; ++i) {
            const double t = (i + 0.5) / nin;
            if (op == 0) x[i] = std::ldexp(1.0 + t, -760 + (int)(t * 1700.0));   // sqrt over [2^-760, 2^940)
            else if (op == 1) x[i] = 0.779 * std::sin(37.0 * t + 0.3);            // |x| < 0.78
            else x[i] = std::ldexp(std::cos(91.0 * t), (int)(t * 40.0) - 20);    // components for a/|a|
        }
        const int nout = nin * width;  // op 2: 6 per vector = 2 per component
        hipError_t e = hipMemcpyAsync(d, x.data(), nin * sizeof(double), hipMemcpyHostToDevice, s);
        if (e == hipSuccess) selftest_math_kernel<<<grid_for(n), kBlock, 0, s>>>(n, d, d + 3 * n, op);
        if (e == hipSuccess) e = hipGetLastError();
        if (e == hipSuccess) e = hipMemcpyAsync(out.data(), d + 3 * n, nout * sizeof(double), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) { st = fail(MOPS_ERR_HIP, std::string("fast-math check: ") + hipGetErrorString(e)); break; }
        // op 0: {fast, lib} per x; op 1: {fast s, lib s, fast c, lib c}; op 2: {3 fast, 3 lib} per vector
        for (int i = 0; i < nout / 2 && st == MOPS_OK; ++i) {
            const int a = (op == 2) ? (i / 3) * 6 + i % 3 : 2 * i, b = (op == 2) ? a + 3 : a + 1;
            if (std::memcmp(&out[a], &out[b], sizeof(double)) != 0)
                st = fail(MOPS_ERR_UNSUPPORTED, "the engine's exact fast-math helpers differ from the device library "
                                                "on this toolchain (bit parity would be lost)");
        }
    }
    (void)hipFree(d);
    return st;
}

extern "C" {

const char* mops_last_error(void) { return g_last_error.c_str(); }
#if defined(MOPS_PROF)
// experiment builds only: read and clear the event counters (dev::g_prof)
int mops_debug_prof(uint64_t* out) {
    unsigned long long h[16];
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(h, HIP_SYMBOL(dev::g_prof), sizeof(h)) != hipSuccess) return -1;
    for (int i = 0; i < 16; ++i) out[i] = h[i];
    const unsigned long long z[16] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(dev::g_prof), z, sizeof(z)) != hipSuccess) return -1;
    return 0;
}
#endif
#if defined(MOPS_WAVE_STAMPS)
// diagnostic builds only: per-slot stamps buffer (device, 4 x u64 per slot) and the
// occupancy API's resident 64-thread blocks per CU of the four MAXV=7 trajectory kernels
int mops_debug_stamps(unsigned long long* d_buf, long long cap, int* occ) {
    if (hipMemcpyToSymbol(HIP_SYMBOL(dev::g_stamps), &d_buf, sizeof(d_buf)) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(dev::g_stamps_cap), &cap, sizeof(cap)) != hipSuccess) return -1;
    if (occ) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[0], traj_kernel<7, false, true>, kTrajBlock, 0) != hipSuccess) return -1;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[1], traj_kernel<7, false, false>, kTrajBlock, 0) != hipSuccess) return -1;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[2], traj_kernel<7, true, true>, kTrajBlock, 0) != hipSuccess) return -1;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ[3], traj_kernel<7, true, false>, kTrajBlock, 0) != hipSuccess) return -1;
    }
    return 0;
}
#endif
int32_t mops_abi_version(void) { return MOPS_ABI_VERSION; }

mops_status mops_selftest_walk(const mops_mesh* mesh, int64_t n, const double* d_pts, const int32_t* d_cells,
                               int32_t* d_out, void* stream) {
    if (!mesh || n < 0 || (n > 0 && (!d_pts || !d_cells || !d_out)))
        return fail(MOPS_ERR_INVALID, "mops_selftest_walk: invalid argument");
    if (!mesh->d_nbr) return fail(MOPS_ERR_UNSUPPORTED, "mops_selftest_walk: no neighbour table (maxEdges > 7)");
    if (n == 0) return MOPS_OK;
    selftest_walk_kernel<<<grid_for(n), kBlock, 0, (hipStream_t)stream>>>(n, d_pts, d_cells, mesh->d_cellrec,
                                                                         mesh->d_cxyz, mesh->d_nbr, (int)mesh->C,
                                                                         d_out);
    HIP_TRY(hipGetLastError());
    return MOPS_OK;
}

mops_status mops_selftest_math(int64_t n, const double* d_x, double* d_out, int32_t op, void* stream) {
    if (n < 0 || (n > 0 && (!d_x || !d_out)) || (op != 0 && op != 1 && op != 2))
        return fail(MOPS_ERR_INVALID, "mops_selftest_math: bad arguments");
    if (n == 0) return MOPS_OK;
    selftest_math_kernel<<<grid_for(n), kBlock, 0, (hipStream_t)stream>>>(n, d_x, d_out, op);
    HIP_TRY(hipGetLastError());
    return MOPS_OK;
}

mops_status mops_mesh_create(const mops_mesh_desc* desc, void* stream, mops_mesh** out) {
    if (!desc || !out) return fail(MOPS_ERR_INVALID, "mops_mesh_create: null argument");
    *out = nullptr;
    const int64_t C = desc->n_cells, V = desc->n_vertices;
    const int maxE = desc->max_edges, L = desc->n_vert_levels;
    if (C <= 0 || V <= 0 || maxE <= 0 || L <= 0 || C >= INT32_MAX || V >= INT32_MAX)
        return fail(MOPS_ERR_INVALID, "mops_mesh_create: invalid sizes");
    if (maxE > kMaxVertex)
        return fail(MOPS_ERR_UNSUPPORTED, "mops_mesh_create: maxEdges > 20 (reference MAX_VERTEX_NUM)");
    // level-pair record indices are 32-bit (dev::pair_sums): V*(L-1) + 1 records < 2^31
    if (V * (int64_t)L >= INT32_MAX)
        return fail(MOPS_ERR_UNSUPPORTED, "mops_mesh_create: nVertices * nVertLevels >= 2^31");
    if (L >= 2 && pr_pieces(V, L) >= ((uint64_t)1 << 32))  // 32-bit record piece indices (pr_base)
        return fail(MOPS_ERR_UNSUPPORTED, "mops_mesh_create: 5 (nVertices + 1) (nVertLevels - 1) >= 2^32");
    if (C > ((int64_t)1 << 30))  // the bucket directory's 32-bit size doubles up to 2C slots
        return fail(MOPS_ERR_UNSUPPORTED, "mops_mesh_create: nCells > 2^30");
    if (MOPS_CPOLY_RANK && maxE <= 7 && C * (int64_t)14 >= ((int64_t)1 << 32))  // d_cpolyr's 32-bit piece index
        return fail(MOPS_ERR_UNSUPPORTED, "mops_mesh_create: 14 nCells >= 2^32 (the cell-rank polygon's 32-bit index)");
    if (!desc->h_n_edges_on_cell || !desc->h_vertices_on_cell || !desc->h_cells_on_cell || !desc->h_cell_coord ||
        !desc->h_vertex_coord)
        return fail(MOPS_ERR_INVALID, "mops_mesh_create: missing mesh array");
    hipStream_t s = (hipStream_t)stream;
    mops_mesh* m = new mops_mesh();
    m->C = C; m->V = V; m->maxE = maxE; m->L = L;
    m->maxv = pick_maxv(maxE);
    m->rec_ints = rec_ints_for(m->maxv);
    // ---- vertex numbering (MOPS_VPERM): the Morton order of the vertex coordinates, so the vertices of
    // neighbouring cells -- the level-pair records one gather instruction asks for -- are close in memory
    std::vector<int> vnew;  // caller's vertex -> internal (empty = identity)
    if (MOPS_VPERM) {
        const double* h = desc->h_vertex_coord;
        std::vector<std::pair<uint64_t, int>> key((size_t)V);
        for (int64_t v = 0; v < V; ++v) key[v] = {vertex_morton_key(h[3 * v], h[3 * v + 1], h[3 * v + 2]), (int)v};
        std::sort(key.begin(), key.end());
        m->h_vold.resize((size_t)V);
        vnew.resize((size_t)V);
        for (int64_t i = 0; i < V; ++i) { m->h_vold[i] = key[i].second; vnew[key[i].second] = (int)i; }
    }
    auto vin = [&](int64_t v) -> int64_t { return vnew.empty() ? v : (int64_t)vnew[v]; };  // caller -> internal
    auto vout = [&](int64_t i) -> int64_t { return m->h_vold.empty() ? i : (int64_t)m->h_vold[i]; };  // internal -> caller
    // ---- cell records (validated) ----
    std::vector<int> rec((size_t)C * m->rec_ints, -1);
    m->h_nv.reserve((size_t)C);
    for (int64_t c = 0; c < C; ++c) {
        const uint64_t ne = desc->h_n_edges_on_cell[c];
        if (ne > (uint64_t)maxE) { free_mesh(m); return fail(MOPS_ERR_INVALID, "nEdgesOnCell > maxEdges"); }
        int* r = rec.data() + c * m->rec_ints;
        r[0] = (int)ne;
        m->h_nv.push_back((int)ne);
        for (int k = 0; k < maxE; ++k) {
            const uint64_t v1 = desc->h_vertices_on_cell[c * maxE + k];
            const uint64_t c1 = desc->h_cells_on_cell[c * maxE + k];
            if (k < (int)ne) {
                if (v1 < 1 || v1 > (uint64_t)V) {
                    free_mesh(m);
                    return fail(MOPS_ERR_INVALID, "verticesOnCell entry out of range for an active edge");
                }
                r[1 + k] = (int)vin((int64_t)(v1 - 1));
            }
            // walk candidates: the reference skips cid < 0 || cid >= C (:910)
            r[1 + m->maxv + k] = (c1 >= 1 && c1 <= (uint64_t)C) ? (int)(c1 - 1) : -1;
        }
    }
    int64_t acc = 0;
    mops_status st;
    if ((st = upload(rec.data(), rec.size(), &m->d_cellrec, &acc, s)) != MOPS_OK) { free_mesh(m); return st; }
    {
        // cell centres + squared "stay" radius rs^2 in .w: rs = half the
        // distance to the nearest valid neighbour centre, shrunk by 1e-9
        // relative and 1 m absolute (>> rounding of |p - c| at Earth radius)
        std::vector<double4> cc((size_t)C);
        const double* h = desc->h_cell_coord;
        for (int64_t c = 0; c < C; ++c) {
            double dmin = INFINITY;
            const int ne = rec[c * m->rec_ints];
            for (int k = 0; k < ne; ++k) {
                const int nb = rec[c * m->rec_ints + 1 + m->maxv + k];
                if (nb < 0) continue;
                const double dx = h[3 * nb] - h[3 * c], dy = h[3 * nb + 1] - h[3 * c + 1], dz = h[3 * nb + 2] - h[3 * c + 2];
                dmin = std::min(dmin, std::sqrt(dx * dx + dy * dy + dz * dz));
            }
            double rs2;
            if (dmin == INFINITY) rs2 = INFINITY;  // no neighbour: the walk can only keep c
            else {
                const double rs = 0.5 * dmin * (1.0 - 1e-9) - 1.0;
                rs2 = (rs > 0.0) ? rs * rs : 0.0;
            }
            cc[c] = make_double4(h[3 * c], h[3 * c + 1], h[3 * c + 2], rs2);
        }
        {   // same arithmetic as locate_kernel's consider() for q = 0: d = -c, sum of squares in dim order
            double best = INFINITY;
            for (int64_t c = 0; c < C; ++c) {
                double dd = 0.0;
                dd += h[3 * c] * h[3 * c]; dd += h[3 * c + 1] * h[3 * c + 1]; dd += h[3 * c + 2] * h[3 * c + 2];
                if (dd < best) { best = dd; m->origin_cell = (int)c; }
            }
        }
        if ((st = dmalloc(&m->d_cxyz, (size_t)C, &acc)) != MOPS_OK) { free_mesh(m); return st; }
        hipError_t e2 = hipMemcpyAsync(m->d_cxyz, cc.data(), C * sizeof(double4), hipMemcpyHostToDevice, s);
        if (e2 == hipSuccess) e2 = hipStreamSynchronize(s);
        if (e2 != hipSuccess) { free_mesh(m); return fail(MOPS_ERR_HIP, hipGetErrorString(e2)); }
    }
    {
        std::vector<double> vc((size_t)V * 3);
        for (int64_t i = 0; i < V; ++i)
            for (int d = 0; d < 3; ++d) vc[3 * i + d] = desc->h_vertex_coord[3 * vout(i) + d];
        if ((st = upload_xyz(vc.data(), V, &m->d_vxyz, &acc, s)) != MOPS_OK) { free_mesh(m); return st; }
    }
    if (!m->h_vold.empty()) {
        if ((st = upload(m->h_vold.data(), m->h_vold.size(), &m->d_vold, &acc, s)) != MOPS_OK) { free_mesh(m); return st; }
    }
    if (desc->h_cells_on_vertex) {
        std::vector<int> cov((size_t)V * 3);
        for (int64_t i = 0; i < V * 3; ++i) {
            const uint64_t x = desc->h_cells_on_vertex[3 * vout(i / 3) + i % 3];
            // reference boundary test: (x - 1) > C + 1 as size_t (Q10); ids C, C+1
            // would read out of range there -- rejected here
            if (x == 0 || x - 1 > (uint64_t)(C + 1)) cov[i] = -1;
            else if (x - 1 >= (uint64_t)C) {
                free_mesh(m);
                return fail(MOPS_ERR_INVALID, "cellsOnVertex entry in [C+1, C+2] (reference reads out of range)");
            } else cov[i] = (int)(x - 1);
        }
        if ((st = upload(cov.data(), cov.size(), &m->d_cov, &acc, s)) != MOPS_OK) { free_mesh(m); return st; }
        if ((st = dmalloc(&m->d_bary, (size_t)V, &acc)) != MOPS_OK) { free_mesh(m); return st; }
        vertex_bary_kernel<<<grid_for(V), kBlock, 0, s>>>(V, m->d_cov, m->d_cxyz, m->d_vxyz, m->d_bary);
    }
    // ---- bucket index for seed location ----
    double rmax = 0.0, rsum = 0.0;
    for (int64_t c = 0; c < C; ++c) {
        const double* p = desc->h_cell_coord + 3 * c;
        const double r = std::sqrt(p[0] * p[0] + p[1] * p[1] + p[2] * p[2]);
        rmax = std::max(rmax, r);
        rsum += r;
    }
    const double rmean = rsum / (double)C;
    const double spacing = std::sqrt(4.0 * M_PI * rmean * rmean / (double)C);
    m->bucket_h = std::max(2.0 * spacing, 1e-9);
    m->bucket_origin = -(rmax * 1.05 + 4.0 * m->bucket_h);
    if ((2.0 * -m->bucket_origin) / m->bucket_h >= (double)((int64_t)1 << 21)) {
        free_mesh(m);
        return fail(MOPS_ERR_UNSUPPORTED, "mesh too fine for the 21-bit bucket grid");
    }
    uint64_t *keys_in = nullptr;
    int* ids_in = nullptr;
    if ((st = dmalloc(&keys_in, (size_t)C, nullptr)) != MOPS_OK) { free_mesh(m); return st; }
    if ((st = dmalloc(&ids_in, (size_t)C, nullptr)) != MOPS_OK) { (void)hipFree(keys_in); free_mesh(m); return st; }
    if ((st = dmalloc(&m->d_bkeys, (size_t)C, &acc)) != MOPS_OK ||
        (st = dmalloc(&m->d_bcells, (size_t)C, &acc)) != MOPS_OK) {
        (void)hipFree(keys_in); (void)hipFree(ids_in); free_mesh(m); return st;
    }
    bucket_keys_kernel<<<grid_for(C), kBlock, 0, s>>>(C, m->d_cxyz, m->bucket_origin, m->bucket_h, keys_in, ids_in);
    size_t tmp_bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, tmp_bytes, keys_in, m->d_bkeys, ids_in, m->d_bcells, (int)C, 0, 63,
                                       s);
    void* tmp = nullptr;
    hipError_t e = hipMalloc(&tmp, std::max<size_t>(tmp_bytes, 1));
    if (e == hipSuccess)
        e = hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys_in, m->d_bkeys, ids_in, m->d_bcells, (int)C, 0, 63,
                                               s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(tmp); (void)hipFree(keys_in); (void)hipFree(ids_in);
    if (e != hipSuccess) { free_mesh(m); return fail(MOPS_ERR_HIP, std::string("bucket sort: ") + hipGetErrorString(e)); }
    {   // Morton rank of every cell (the particles' locality key): one sort of the centres' keys
        uint64_t *ck = nullptr, *ck_sorted = nullptr;
        int *cid = nullptr, *cid_sorted = nullptr;
        void* ctmp = nullptr;
        size_t ctmp_bytes = 0;
        e = hipcub::DeviceRadixSort::SortPairs(nullptr, ctmp_bytes, ck, ck_sorted, cid, cid_sorted, (int)C, 0, 63, s);
        if (e == hipSuccess) e = hipMalloc(&ck, (size_t)C * sizeof(uint64_t));
        if (e == hipSuccess) e = hipMalloc(&ck_sorted, (size_t)C * sizeof(uint64_t));
        if (e == hipSuccess) e = hipMalloc(&cid, (size_t)C * sizeof(int));
        if (e == hipSuccess) e = hipMalloc(&cid_sorted, (size_t)C * sizeof(int));
        if (e == hipSuccess) e = hipMalloc(&ctmp, std::max<size_t>(ctmp_bytes, 1));
        if (e == hipSuccess && (st = dmalloc(&m->d_cell_rank, (size_t)C, &acc)) != MOPS_OK) e = hipErrorOutOfMemory;
        if (e == hipSuccess) {
            cell_key_kernel<<<grid_for(C), kBlock, 0, s>>>(C, m->d_cxyz, ck, cid);
            e = hipcub::DeviceRadixSort::SortPairs(ctmp, ctmp_bytes, ck, ck_sorted, cid, cid_sorted, (int)C, 0, 63, s);
        }
        if (e == hipSuccess) {
            cell_rank_kernel<<<grid_for(C), kBlock, 0, s>>>(C, cid_sorted, m->d_cell_rank);
            e = hipStreamSynchronize(s);
        }
        (void)hipFree(ck); (void)hipFree(ck_sorted); (void)hipFree(cid); (void)hipFree(ctmp);
        m->d_rank_cell = cid_sorted;  // kept: the cell of each rank (cpoly_rank_kernel)
        acc += C * (int64_t)sizeof(int);
        if (e != hipSuccess) { free_mesh(m); return fail(MOPS_ERR_HIP, std::string("cell rank sort: ") + hipGetErrorString(e)); }
    }
    if ((st = dmalloc(&m->d_rloc2, (size_t)C, &acc)) != MOPS_OK) { free_mesh(m); return st; }
    if ((st = dmalloc(&m->d_ring, (size_t)C, &acc)) != MOPS_OK) { free_mesh(m); return st; }
    {   // bucket directory (BucketDir): H = 2^k >= 2 C slots, so it is at most half full
        uint32_t H = 2;
        while ((int64_t)H < 2 * C) H <<= 1;
        m->hmask = H - 1;
        if ((st = dmalloc(&m->d_hkeys, (size_t)H, &acc)) != MOPS_OK ||
            (st = dmalloc(&m->d_hval, (size_t)H, &acc)) != MOPS_OK) { free_mesh(m); return st; }
        e = hipMemsetAsync(m->d_hkeys, 0xff, (size_t)H * sizeof(uint64_t), s);  // kEmptyKey
        if (e != hipSuccess) { free_mesh(m); return fail(MOPS_ERR_HIP, hipGetErrorString(e)); }
        bucket_dir_kernel<<<grid_for(C), kBlock, 0, s>>>(C, m->d_bkeys, m->d_hkeys, m->d_hval, m->hmask);
    }
    locate_radius_kernel<<<grid_for(C), kBlock, 0, s>>>(C, m->d_cxyz, bucket_dir(m), m->bucket_origin,
                                                        m->bucket_h, m->d_cellrec, m->rec_ints, m->maxv,
                                                        m->d_rloc2, m->d_ring);
    if ((st = dmalloc(&m->d_cpoly, (size_t)(C * m->maxv), &acc)) != MOPS_OK) { free_mesh(m); return st; }
    if (m->maxv == 7 && (st = dmalloc(&m->d_cnrm, (size_t)(C * kCellNrm), &acc)) != MOPS_OK) { free_mesh(m); return st; }
    if (MOPS_TILE_E1 && m->maxv == 7 && (st = dmalloc(&m->d_cedge, (size_t)(C * kCellNrm), &acc)) != MOPS_OK) {
        free_mesh(m);
        return st;
    }
    if (m->maxv == 7 && (st = dmalloc(&m->d_nbr, (size_t)(C * kNbrQ), &acc)) != MOPS_OK) { free_mesh(m); return st; }
    if (m->maxv == 7) cell_nbr_kernel<<<grid_for(C), kBlock, 0, s>>>(C, m->d_cellrec, m->d_cxyz, m->d_nbr);
    switch (m->maxv) {
        case 7:
            cell_poly_kernel<7><<<grid_for(C), kBlock, 0, s>>>(C, m->d_cellrec, m->d_vxyz, m->d_cpoly, m->d_cnrm, m->d_cedge);
            if (MOPS_CPOLY_RANK) {
                if ((st = dmalloc(&m->d_cpolyr, (size_t)(C * 14), &acc)) != MOPS_OK) { free_mesh(m); return st; }
                cpoly_rank_kernel<<<grid_for(C * 14), kBlock, 0, s>>>(C, m->d_rank_cell, m->d_cpoly, m->d_cpolyr);
            }
            break;
        case 12: cell_poly_kernel<12><<<grid_for(C), kBlock, 0, s>>>(C, m->d_cellrec, m->d_vxyz, m->d_cpoly); break;
        default: cell_poly_kernel<20><<<grid_for(C), kBlock, 0, s>>>(C, m->d_cellrec, m->d_vxyz, m->d_cpoly); break;
    }
    e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    if (e != hipSuccess) { free_mesh(m); return fail(MOPS_ERR_HIP, std::string("cell keys: ") + hipGetErrorString(e)); }
    if ((st = check_fast_math(s)) != MOPS_OK) { free_mesh(m); return st; }
    m->bytes = acc;
    *out = m;
    return MOPS_OK;
}

void mops_mesh_destroy(mops_mesh* mesh) { free_mesh(mesh); }
int64_t mops_mesh_bytes(const mops_mesh* mesh) { return mesh ? mesh->bytes : 0; }

mops_status mops_mesh_set_edges(mops_mesh* m, int64_t n_edges, const uint64_t* h_edges_on_cell,
                                const uint64_t* h_cells_on_edge, const double* h_edge_coord, void* stream) {
    if (!m || n_edges <= 0 || n_edges >= INT32_MAX || !h_edges_on_cell || !h_cells_on_edge || !h_edge_coord)
        return fail(MOPS_ERR_INVALID, "mops_mesh_set_edges: invalid argument");
    if (m->d_eoc) return fail(MOPS_ERR_INVALID, "mops_mesh_set_edges: the mesh already has edges");
    const int64_t C = m->C, E = n_edges;
    const int maxE = m->maxE;
    // cellsOnEdge, 0-based; -1 = the reference's "max_cell_id > CELL_SIZE" side (id 0, or id - 1 > C)
    std::vector<int2> coe((size_t)E);
    for (int64_t e = 0; e < E; ++e) {
        int v[2];
        for (int j = 0; j < 2; ++j) {
            const uint64_t x = h_cells_on_edge[2 * e + j];
            if (x >= 1 && x <= (uint64_t)C) v[j] = (int)(x - 1);
            else if (x == (uint64_t)C + 1) return fail(MOPS_ERR_INVALID, "cellsOnEdge entry C+1 (reference reads out of range)");
            else v[j] = -1;
        }
        coe[(size_t)e] = make_int2(v[0], v[1]);
    }
    std::vector<int> eoc((size_t)C * kRbfN, -1);
    for (int64_t c = 0; c < C; ++c) {
        const int nv = m->h_nv[(size_t)c];
        if (nv > kRbfN)
            return fail(MOPS_ERR_UNSUPPORTED, "mops_mesh_set_edges: a cell with more than 7 edges (the reference's RBF "
                                              "stencil holds MAX_VERTEX_NUM = 7, MPASOSolutionTBB.cpp:142)");
        for (int k = 0; k < nv; ++k) {
            const uint64_t x = h_edges_on_cell[c * maxE + k];
            if (x == 0) continue;  // the reference skips it (edge id SIZE_MAX)
            if (x > (uint64_t)E) return fail(MOPS_ERR_INVALID, "edgesOnCell entry out of range");
            const int e = (int)(x - 1);
            if (coe[(size_t)e].x < 0 && coe[(size_t)e].y < 0)
                return fail(MOPS_ERR_INVALID, "an edge of a cell has no valid cellsOnEdge entry (reference reads "
                                              "cellCoord[SIZE_MAX])");
            eoc[(size_t)(c * kRbfN + k)] = e;
        }
    }
    hipStream_t s = (hipStream_t)stream;
    int64_t acc = 0;
    mops_status st;
    if ((st = upload(eoc.data(), eoc.size(), &m->d_eoc, &acc, s)) != MOPS_OK ||
        (st = upload(coe.data(), coe.size(), &m->d_coe, &acc, s)) != MOPS_OK ||
        (st = upload_xyz(h_edge_coord, E, &m->d_exyz, &acc, s)) != MOPS_OK ||
        (st = dmalloc(&m->d_rbf_coef, (size_t)(C * kRbfN * 3), &acc)) != MOPS_OK ||
        (st = dmalloc(&m->d_rbf_slot, (size_t)(C * kRbfN), &acc)) != MOPS_OK) {
        (void)hipFree(m->d_eoc); (void)hipFree(m->d_coe); (void)hipFree(m->d_exyz); (void)hipFree(m->d_rbf_coef);
        (void)hipFree(m->d_rbf_slot);
        m->d_eoc = nullptr; m->d_coe = nullptr; m->d_exyz = nullptr; m->d_rbf_coef = nullptr; m->d_rbf_slot = nullptr;
        return st;
    }
    rbf_coef_kernel<<<(unsigned)((C + 63) / 64), 64, 0, s>>>(C, m->rec_ints, m->d_cellrec, m->d_eoc, m->d_coe,
                                                             m->d_exyz, m->d_cxyz, m->d_rbf_coef, m->d_rbf_slot);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipStreamSynchronize(s));
    m->E = E;
    m->bytes += acc;
    return MOPS_OK;
}

mops_status mops_cell_center_velocity_rbf(const mops_mesh* m, const double* d_normal_velocity, double* d_out,
                                          void* stream) {
    if (!m || !d_normal_velocity || !d_out) return fail(MOPS_ERR_INVALID, "mops_cell_center_velocity_rbf: null argument");
    if (!m->d_rbf_coef) return fail(MOPS_ERR_INVALID, "mops_cell_center_velocity_rbf: the mesh has no edges "
                                                      "(mops_mesh_set_edges)");
    const int64_t n = m->C * (int64_t)m->L;
    rbf_apply_kernel<<<grid_for(n), kBlock, 0, (hipStream_t)stream>>>(m->C, m->L, m->d_rbf_coef, m->d_rbf_slot,
                                                                      d_normal_velocity, d_out);
    HIP_TRY(hipGetLastError());
    return MOPS_OK;
}

// the all-zero record's pieces (pair_sums reads it for slots v >= nv): vertex V of every (layer, piece) row
// (piece-major) or the record after the last (record-major); the builders never write them
__global__ void pr_zero_kernel(int64_t V, int L, double2* __restrict__ pr) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (MOPS_PR_PIECES) {
        if (i < (int64_t)(L - 1) * (kPairRec / 2)) pr[(uint64_t)i * (uint64_t)(V + 1) + (uint64_t)V] = make_double2(0.0, 0.0);
    } else if (i < kPairRec / 2) {
        pr[pr_zero((uint32_t)V, (uint32_t)L) + (uint32_t)i] = make_double2(0.0, 0.0);
    }
}

static mops_status alloc_records(const mops_mesh* mesh, mops_field* f, hipStream_t s) {
    if (mesh->L < 2) return MOPS_OK;
    if (!f->d_pr) MOPS_TRY(dmalloc(&f->d_pr, (size_t)(pr_pieces(mesh->V, mesh->L) * 2), &f->bytes));
    pr_zero_kernel<<<grid_for((int64_t)(mesh->L - 1) * (kPairRec / 2)), kBlock, 0, s>>>(
        mesh->V, mesh->L, reinterpret_cast<double2*>(f->d_pr));
    HIP_TRY(hipGetLastError());
    return MOPS_OK;
}

static mops_status compute_flags(const mops_mesh* mesh, mops_field* f, hipStream_t s);

// records from the vertex arrays (fields uploaded as vertex arrays), then the fast-path flags
static mops_status compute_mono(const mops_mesh* mesh, mops_field* f, hipStream_t s) {
    const int64_t npr = mesh->V * (int64_t)std::max(mesh->L - 1, 0);
    MOPS_TRY(alloc_records(mesh, f, s));
#if MOPS_REC_TILED
    if (npr > 0) {
        const dim3 grid((unsigned)((mesh->V + kRecTV - 1) / kRecTV), (unsigned)((mesh->L - 1 + kRecTK - 1) / kRecTK));
        pair_record_tiled_kernel<<<grid, 256, 0, s>>>(mesh->V, mesh->L, f->d_zt, f->d_vel, f->d_w, f->d_pr);
    }
#else
    if (npr > 0)
    {
        const int64_t chunks = npr * (kPairRec / 2);
        if (chunks < ((int64_t)1 << 32) - kBlock)
            pair_record_kernel<uint32_t><<<grid_for(chunks), kBlock, 0, s>>>(mesh->V, mesh->L, f->d_zt, f->d_vel,
                                                                           f->d_w, f->d_pr);
        else
            pair_record_kernel<uint64_t><<<grid_for(chunks), kBlock, 0, s>>>(mesh->V, mesh->L, f->d_zt, f->d_vel,
                                                                           f->d_w, f->d_pr);
    }
#endif
    return compute_flags(mesh, f, s);
}

static mops_status compute_flags(const mops_mesh* mesh, mops_field* f, hipStream_t s) {
    if (!f->d_mono) MOPS_TRY(dmalloc(&f->d_mono, (size_t)mesh->C, &f->bytes));
    if (!f->d_vmono) MOPS_TRY(dmalloc(&f->d_vmono, (size_t)mesh->V, &f->bytes));
    if (!f->d_vzero) MOPS_TRY(dmalloc(&f->d_vzero, (size_t)mesh->V, &f->bytes));
    fill_i32_kernel<<<grid_for(mesh->V), kBlock, 0, s>>>(mesh->V, mesh->L, f->d_vmono);
    HIP_TRY(hipMemsetAsync(f->d_vzero, 1, (size_t)mesh->V, s));
    vertex_mono_kernel<<<grid_for(mesh->V * mesh->L), kBlock, 0, s>>>(mesh->V, mesh->L, f->d_zt, f->d_vmono,
                                                                      f->d_vzero);
    mono_kernel<<<grid_for(mesh->C), kBlock, 0, s>>>(mesh->C, mesh->maxv, mesh->rec_ints, mesh->d_cellrec, f->d_vmono,
                                                    f->d_vzero, mesh->L, f->d_mono);
    HIP_TRY(hipGetLastError());
    return MOPS_OK;
}

mops_status mops_field_create_derived(const mops_mesh* mesh, const double* h_zt, const double* h_vel,
                                      const double* h_w, void* stream, mops_field** out) {
    if (!mesh || !out || !h_zt || !h_vel) return fail(MOPS_ERR_INVALID, "mops_field_create_derived: null argument");
    *out = nullptr;
    hipStream_t s = (hipStream_t)stream;
    mops_field* f = new mops_field();
    f->mesh = mesh; f->V = mesh->V; f->L = mesh->L;
    const size_t V = (size_t)mesh->V, L = (size_t)mesh->L;
    mops_status st;
    // the caller's vertex rows in the internal vertex order (mops_mesh::h_vold)
    std::vector<double> pzt, pvel, pw;
    if (!mesh->h_vold.empty()) {
        auto perm = [&](const double* src, size_t row, std::vector<double>& dst) {
            dst.resize(V * row);
            for (size_t i = 0; i < V; ++i)
                std::memcpy(dst.data() + i * row, src + (size_t)mesh->h_vold[i] * row, row * sizeof(double));
            return dst.data();
        };
        h_zt = perm(h_zt, L, pzt);
        h_vel = perm(h_vel, L * 3, pvel);
        if (h_w) h_w = perm(h_w, L + 1, pw);
    }
    if ((st = upload(h_zt, V * L, &f->d_zt, &f->bytes, s)) != MOPS_OK ||
        (st = upload(h_vel, V * L * 3, &f->d_vel, &f->bytes, s)) != MOPS_OK) { free_field(f); return st; }
    if (h_w) {
        if ((st = upload(h_w, V * (L + 1), &f->d_w, &f->bytes, s)) != MOPS_OK) { free_field(f); return st; }
    } else {
        if ((st = dmalloc(&f->d_w, V * (L + 1), &f->bytes)) != MOPS_OK) { free_field(f); return st; }
        HIP_TRY(hipMemsetAsync(f->d_w, 0, V * (L + 1) * sizeof(double), s));
    }
    if ((st = compute_mono(mesh, f, s)) != MOPS_OK) { free_field(f); return st; }
    HIP_TRY(hipStreamSynchronize(s));
    *out = f;
    return MOPS_OK;
}

static mops_status field_create_impl(const mops_mesh* mesh, const mops_snapshot_desc* desc, bool on_device,
                                     hipStream_t s, mops_field** out);
static mops_status field_derive(const mops_mesh* mesh, mops_field* f, const mops_snapshot_desc* d, double* ztc,
                                double* velc, hipStream_t s);

mops_status mops_field_create(const mops_mesh* mesh, const mops_snapshot_desc* desc, void* stream,
                              mops_field** out) {
    return field_create_impl(mesh, desc, false, (hipStream_t)stream, out);
}

mops_status mops_field_create_device(const mops_mesh* mesh, const mops_snapshot_desc* d_desc, void* stream,
                                     mops_field** out) {
    return field_create_impl(mesh, d_desc, true, (hipStream_t)stream, out);
}

mops_status mops_field_rebuild_device(mops_field* field, const mops_snapshot_desc* d_desc, void* stream) {
    if (!field || !d_desc || !field->mesh) return fail(MOPS_ERR_INVALID, "mops_field_rebuild_device: null argument");
    if (!field->d_ztc || !field->d_velc)
        return fail(MOPS_ERR_INVALID, "mops_field_rebuild_device: field was not created by mops_field_create_device");
    return field_derive(field->mesh, field, d_desc, field->d_ztc, field->d_velc, (hipStream_t)stream);
}

}  // extern "C"

static mops_status check_snapshot(const mops_mesh* mesh, const mops_snapshot_desc* desc) {
    if (!desc->h_layer_thickness)
        return fail(MOPS_ERR_INVALID, "cellLayerThickness is not defined");  // MPASOSolution.cpp:540-544
    const bool zm = desc->h_zonal_velocity && desc->h_meridional_velocity;
    if (!zm && !(desc->h_normal_velocity && mesh->d_rbf_coef))
        return fail(MOPS_ERR_INVALID, "zonal/meridional velocity (or normalVelocity on a mesh with edges) required");
    if (!mesh->d_cov) return fail(MOPS_ERR_INVALID, "mesh has no cellsOnVertex");
    return MOPS_OK;
}

// Enqueue the derivation chain (MOPSApp::addSol: calcCellCenterZtop, CalcCellVertexZtop,
// CalcCellCenterVelocityByZM, CalcCellVertexVelocity, CalcCellVertexVertVelocity, then the
// engine's level-pair records and monotone flags) from raw DEVICE arrays `d` into f,
// allocating only the buffers f does not have yet.  Asynchronous on s.
static mops_status field_derive(const mops_mesh* mesh, mops_field* f, const mops_snapshot_desc* d, double* ztc,
                                double* velc, hipStream_t s) {
    MOPS_TRY(check_snapshot(mesh, d));
    const int64_t C = mesh->C, V = mesh->V;
    const int L = mesh->L;
    const double* bot = d->h_bottom_depth;
    const double* ssh = bot ? nullptr : d->h_surface_height;
    if (!f->d_zt) MOPS_TRY(dmalloc(&f->d_zt, (size_t)(V * L), &f->bytes));
    if (!f->d_vel) MOPS_TRY(dmalloc(&f->d_vel, (size_t)(V * L * 3), &f->bytes));
    if (!f->d_w) MOPS_TRY(dmalloc(&f->d_w, (size_t)(V * (L + 1)), &f->bytes));
    cell_ztop_tiled_kernel<<<(unsigned)((C + kZtCells - 1) / kZtCells), 256, (size_t)kZtCells * L * sizeof(double), s>>>(
        C, L, d->h_layer_thickness, bot, ssh, ztc);
    if (d->h_zonal_velocity && d->h_meridional_velocity) {  // the live path (MOPSApp.cpp:113)
        center_vel_zm_kernel<<<grid_for(C * L), kBlock, 0, s>>>(C, L, mesh->d_cxyz, d->h_zonal_velocity,
                                                                d->h_meridional_velocity, velc);
    } else {  // edge normals only: the RBF reconstruction (MPASOSolution::calcCellCenterVelocity)
        MOPS_TRY(mops_cell_center_velocity_rbf(mesh, d->h_normal_velocity, velc, s));
    }
#if MOPS_FUSED_RECORDS
    if (L >= 2) {
        // CalcCellVertexZtop / CalcCellVertexVelocity / CalcCellVertexVertVelocity fused into the
        // level-pair record build (pair_record_fused_kernel)
        MOPS_TRY(alloc_records(mesh, f, s));
        const dim3 grid((unsigned)((V + kRecTV - 1) / kRecTV), (unsigned)((L - 1 + kRecTK - 1) / kRecTK));
        if (d->h_vert_velocity_top)
            pair_record_fused_kernel<true><<<grid, 256, 0, s>>>(V, L, mesh->d_cov, mesh->d_bary, ztc, velc,
                                                                d->h_vert_velocity_top, f->d_zt, f->d_w, f->d_pr);
        else
            pair_record_fused_kernel<false><<<grid, 256, 0, s>>>(V, L, mesh->d_cov, mesh->d_bary, ztc, velc, nullptr,
                                                                 f->d_zt, f->d_w, f->d_pr);
        f->vtx_full = false;
        MOPS_TRY(compute_flags(mesh, f, s));
        HIP_TRY(hipGetLastError());
        return MOPS_OK;
    }
#endif
    cell_to_vertex_bary_kernel<1><<<grid_for(V * L), kBlock, 0, s>>>(V, L, mesh->d_cov, mesh->d_bary, ztc, f->d_zt, 0);
    cell_to_vertex_bary_kernel<3><<<grid_for(V * L), kBlock, 0, s>>>(V, L, mesh->d_cov, mesh->d_bary, velc, f->d_vel, 0);
    if (d->h_vert_velocity_top) {
        cell_to_vertex_bary_kernel<1><<<grid_for(V * (L + 1)), kBlock, 0, s>>>(V, L + 1, mesh->d_cov, mesh->d_bary,
                                                                              d->h_vert_velocity_top, f->d_w, 0);
    } else {
        HIP_TRY(hipMemsetAsync(f->d_w, 0, (size_t)(V * (L + 1)) * sizeof(double), s));
    }
    MOPS_TRY(compute_mono(mesh, f, s));
    HIP_TRY(hipGetLastError());
    return MOPS_OK;
}

// Raw inputs either uploaded from host (mops_field_create: staged, then freed) or
// read in place from HBM (mops_field_create_device: nothing copied; the
// intermediates are kept for mops_field_rebuild_device).
static mops_status field_create_impl(const mops_mesh* mesh, const mops_snapshot_desc* desc, bool on_device,
                                     hipStream_t s, mops_field** out) {
    if (!mesh || !desc || !out) return fail(MOPS_ERR_INVALID, "mops_field_create: null argument");
    *out = nullptr;
    MOPS_TRY(check_snapshot(mesh, desc));
    const int64_t C = mesh->C;
    const int L = mesh->L;
    mops_field* f = new mops_field();
    f->mesh = mesh; f->V = mesh->V; f->L = L;
    mops_snapshot_desc dd = *desc;  // device view of the raw arrays
    double *thick = nullptr, *bot = nullptr, *ssh = nullptr, *zon = nullptr, *mer = nullptr, *wc = nullptr;
    double* nrm = nullptr;
    double *ztc = nullptr, *velc = nullptr;
    int64_t scratch = 0;
    mops_status st = MOPS_OK;
    do {
        if (!on_device) {
            if ((st = upload(desc->h_layer_thickness, (size_t)(C * L), &thick, &scratch, s)) != MOPS_OK) break;
            if (desc->h_bottom_depth && (st = upload(desc->h_bottom_depth, (size_t)C, &bot, &scratch, s)) != MOPS_OK)
                break;
            if (!desc->h_bottom_depth && desc->h_surface_height &&
                (st = upload(desc->h_surface_height, (size_t)C, &ssh, &scratch, s)) != MOPS_OK) break;
            if (desc->h_zonal_velocity && desc->h_meridional_velocity) {
                if ((st = upload(desc->h_zonal_velocity, (size_t)(C * L), &zon, &scratch, s)) != MOPS_OK) break;
                if ((st = upload(desc->h_meridional_velocity, (size_t)(C * L), &mer, &scratch, s)) != MOPS_OK) break;
            } else if ((st = upload(desc->h_normal_velocity, (size_t)(mesh->E * L), &nrm, &scratch, s)) != MOPS_OK) {
                break;
            }
            if (desc->h_vert_velocity_top &&
                (st = upload(desc->h_vert_velocity_top, (size_t)(C * (L + 1)), &wc, &scratch, s)) != MOPS_OK) break;
            dd.h_layer_thickness = thick; dd.h_bottom_depth = bot; dd.h_surface_height = ssh;
            dd.h_zonal_velocity = zon; dd.h_meridional_velocity = mer; dd.h_vert_velocity_top = wc;
            dd.h_normal_velocity = nrm;
        }
        if ((st = dmalloc(&ztc, (size_t)(C * L), on_device ? &f->bytes : &scratch)) != MOPS_OK) break;
        if (on_device) f->d_ztc = ztc;  // owned by the field from here on
        if ((st = dmalloc(&velc, (size_t)(C * L * 3), on_device ? &f->bytes : &scratch)) != MOPS_OK) break;
        if (on_device) f->d_velc = velc;
        if ((st = field_derive(mesh, f, &dd, ztc, velc, s)) != MOPS_OK) break;
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) { st = fail(MOPS_ERR_HIP, std::string("preprocessing: ") + hipGetErrorString(e)); break; }
    } while (0);
    if (!on_device) {
        (void)hipFree(thick); (void)hipFree(bot); (void)hipFree(ssh); (void)hipFree(zon); (void)hipFree(mer);
        (void)hipFree(wc); (void)hipFree(nrm); (void)hipFree(ztc); (void)hipFree(velc);
    }
    if (st != MOPS_OK) { free_field(f); return st; }
    *out = f;
    return MOPS_OK;
}

extern "C" {

mops_status mops_cell_to_vertex_attr(const mops_mesh* mesh, const double* d_cell_attr, double* d_vertex_attr,
                                     void* stream) {
    if (!mesh || !d_cell_attr || !d_vertex_attr || !mesh->d_cov)
        return fail(MOPS_ERR_INVALID, "mops_cell_to_vertex_attr: null argument");
    hipStream_t s = (hipStream_t)stream;
    cell_to_vertex_bary_kernel<1><<<grid_for(mesh->V * mesh->L), kBlock, 0, s>>>(
        mesh->V, mesh->L, mesh->d_cov, mesh->d_bary, d_cell_attr, d_vertex_attr, 1, mesh->d_vold);
    HIP_TRY(hipGetLastError());
    return MOPS_OK;
}

mops_status mops_field_export(const mops_field* f, double* h_zt, double* h_vel, double* h_w, void* stream) {
    if (!f) return fail(MOPS_ERR_INVALID, "mops_field_export: null field");
    hipStream_t s = (hipStream_t)stream;
    const size_t V = (size_t)f->V, L = (size_t)f->L;
    if (h_zt) HIP_TRY(hipMemcpyAsync(h_zt, f->d_zt, V * L * sizeof(double), hipMemcpyDeviceToHost, s));
    if ((h_vel || h_w) && !f->vtx_full && L >= 2)  // fused field: rebuild the vertex arrays from the records
        records_to_vertex_kernel<<<grid_for((int64_t)(V * L)), kBlock, 0, s>>>((int64_t)V, (int)L, f->d_pr, f->d_vel,
                                                                               f->d_w);
    if (h_vel) HIP_TRY(hipMemcpyAsync(h_vel, f->d_vel, V * L * 3 * sizeof(double), hipMemcpyDeviceToHost, s));
    if (h_w) HIP_TRY(hipMemcpyAsync(h_w, f->d_w, V * (L + 1) * sizeof(double), hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    const std::vector<int>& vold = f->mesh->h_vold;  // internal rows -> the caller's vertex order
    if (!vold.empty()) {
        std::vector<double> tmp;
        auto unperm = [&](double* buf, size_t row) {
            tmp.assign(buf, buf + V * row);
            for (size_t i = 0; i < V; ++i)
                std::memcpy(buf + (size_t)vold[i] * row, tmp.data() + i * row, row * sizeof(double));
        };
        if (h_zt) unperm(h_zt, L);
        if (h_vel) unperm(h_vel, L * 3);
        if (h_w) unperm(h_w, L + 1);
    }
    return MOPS_OK;
}

void mops_field_destroy(mops_field* field) { free_field(field); }
int64_t mops_field_bytes(const mops_field* field) { return field ? field->bytes : 0; }

mops_status mops_locate_cells(const mops_mesh* mesh, int64_t n, const double* d_points, int32_t* d_cells,
                              void* stream) {
    if (!mesh || n < 0 || (n > 0 && (!d_points || !d_cells)))
        return fail(MOPS_ERR_INVALID, "mops_locate_cells: invalid argument");
    if (n == 0) return MOPS_OK;
    hipStream_t s = (hipStream_t)stream;
    locate_kernel<<<grid_for(n), kBlock, 0, s>>>(n, d_points, mesh->C, mesh->d_cxyz, bucket_dir(mesh),
                                                 mesh->bucket_origin, mesh->bucket_h, mesh->origin_cell, nullptr,
                                                 nullptr, nullptr, nullptr, 0, 0, d_cells);
    HIP_TRY(hipGetLastError());
    return MOPS_OK;
}

mops_status mops_locate_cells_hinted(const mops_mesh* mesh, int64_t n, const double* d_points, const int32_t* d_hint,
                                     int32_t* d_cells, void* stream) {
    if (!mesh || n < 0 || (n > 0 && (!d_points || !d_cells)))
        return fail(MOPS_ERR_INVALID, "mops_locate_cells_hinted: invalid argument");
    if (n == 0) return MOPS_OK;
    hipStream_t s = (hipStream_t)stream;
    locate_kernel<<<grid_for(n), kBlock, 0, s>>>(n, d_points, mesh->C, mesh->d_cxyz, bucket_dir(mesh),
                                                 mesh->bucket_origin, mesh->bucket_h, mesh->origin_cell, d_hint,
                                                 mesh->d_rloc2, mesh->d_ring, mesh->d_cellrec, mesh->rec_ints,
                                                 mesh->maxv, d_cells);
    HIP_TRY(hipGetLastError());
    return MOPS_OK;
}

// Scratch of the particle locality sort, 256-B aligned parts: keys in, keys out, slot index in,
// then hipcub's radix temp (sized for all 32 key bits, which covers any particle_key_bits)
struct OrderScratch {
    size_t a4 = 0, tmp_bytes = 0, need = 0;
};
static hipError_t order_scratch_layout(int64_t n, OrderScratch& o) {
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, o.tmp_bytes, (const uint32_t*)nullptr,
                                                      (uint32_t*)nullptr, (const int*)nullptr, (int*)nullptr, (int)n,
                                                      0, 32, (hipStream_t)0);
    o.a4 = ((size_t)n * 4 + 255) / 256 * 256;
    o.need = 3 * o.a4 + o.tmp_bytes + 256;  // (+ alignment slack for a caller's buffer)
    return e;
}
static mops_status order_sort(const mops_mesh* mesh, int64_t n, const int32_t* d_cell, const int32_t* d_death,
                              int32_t* d_order, int32_t* d_n_live, void* scratch, const OrderScratch& o,
                              hipStream_t s) {
    char* base = (char*)(((uintptr_t)scratch + 255) / 256 * 256);
    uint32_t* kin = (uint32_t*)base;
    uint32_t* kout = (uint32_t*)(base + o.a4);
    int* vin = (int*)(base + 2 * o.a4);
    void* tmp = base + 3 * o.a4;
    if (d_n_live) HIP_TRY(hipMemsetAsync(d_n_live, 0, sizeof(int32_t), s));
    particle_key_kernel<<<grid_for(n), kBlock, 0, s>>>(n, mesh->C, d_cell, d_death, mesh->d_cell_rank, kin, vin,
                                                       d_n_live);
    HIP_TRY(hipGetLastError());
    size_t tb = o.tmp_bytes;
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(tmp, tb, kin, kout, vin, d_order, (int)n, 0,
                                               particle_key_bits(mesh->C), s));
    return MOPS_OK;
}

mops_status mops_order_particles(const mops_mesh* mesh, int64_t n, const int32_t* d_cell, int32_t* d_order,
                                 void* stream) {
    if (!mesh || n < 0 || (n > 0 && (!d_cell || !d_order)) || n >= INT32_MAX)
        return fail(MOPS_ERR_INVALID, "mops_order_particles: invalid argument");
    if (n == 0) return MOPS_OK;
    hipStream_t s = (hipStream_t)stream;
    OrderScratch o;
    HIP_TRY(order_scratch_layout(n, o));
    if (mesh->scratch_bytes < o.need) {
        HIP_TRY(hipStreamSynchronize(s));
        (void)hipFree(mesh->d_scratch);
        mesh->d_scratch = nullptr;
        mesh->scratch_bytes = 0;
        HIP_TRY(hipMalloc(&mesh->d_scratch, o.need));
        mesh->scratch_bytes = o.need;
    }
    return order_sort(mesh, n, d_cell, nullptr, d_order, nullptr, mesh->d_scratch, o, s);
}

int64_t mops_order_scratch_bytes(int64_t n) {
    if (n <= 0 || n >= INT32_MAX) return 0;
    OrderScratch o;
    if (order_scratch_layout(n, o) != hipSuccess) return 0;
    return (int64_t)o.need;
}

mops_status mops_permute_arrays(int64_t n, const int32_t* d_order, int32_t count, const mops_perm_array* arrays,
                                void* stream) {
    if (n < 0 || count < 0 || count > kPermMax || (count > 0 && !arrays))
        return fail(MOPS_ERR_INVALID, "mops_permute_arrays: invalid argument");
    if (n == 0 || count == 0) return MOPS_OK;
    PermArrays a{};
    a.count = count;
    int rows = 0;
    for (int k = 0; k < count; ++k) {
        const mops_perm_array& d = arrays[k];
        if (!d.d_src || !d.d_dst || (d.elem_bytes != 4 && d.elem_bytes != 8 && d.elem_bytes != 24) || d.rows < 1 ||
            (d.rows > 1 && d.row_stride < n) || d.d_src == d.d_dst)
            return fail(MOPS_ERR_INVALID, "mops_permute_arrays: bad array descriptor (out of place, 4/8/24-B elements)");
        a.src[k] = static_cast<const char*>(d.d_src);
        a.dst[k] = static_cast<char*>(d.d_dst);
        a.elem[k] = (int)d.elem_bytes;
        a.stride_bytes[k] = d.row_stride * d.elem_bytes;
        a.row0[k] = rows;
        rows += (int)d.rows;
        if (rows > 65535) return fail(MOPS_ERR_INVALID, "mops_permute_arrays: more than 65535 rows");
    }
    a.row0[count] = rows;
    const dim3 grid((unsigned)((n + kBlock - 1) / kBlock), (unsigned)rows);
    permute_kernel<<<grid, kBlock, 0, (hipStream_t)stream>>>(n, d_order, a);
    HIP_TRY(hipGetLastError());
    return MOPS_OK;
}

mops_status mops_order_particles_live(const mops_mesh* mesh, int64_t n, const int32_t* d_cell, const int32_t* d_death,
                                      int32_t* d_order, int32_t* d_n_live, void* d_scratch, int64_t scratch_bytes,
                                      void* stream) {
    if (!mesh || n < 0 || (n > 0 && (!d_cell || !d_order || !d_scratch)) || n >= INT32_MAX)
        return fail(MOPS_ERR_INVALID, "mops_order_particles_live: invalid argument");
    if (n == 0) {
        if (d_n_live) HIP_TRY(hipMemsetAsync(d_n_live, 0, sizeof(int32_t), (hipStream_t)stream));
        return MOPS_OK;
    }
    OrderScratch o;
    HIP_TRY(order_scratch_layout(n, o));
    if (scratch_bytes < (int64_t)o.need)
        return fail(MOPS_ERR_INVALID, "mops_order_particles_live: scratch smaller than mops_order_scratch_bytes(n)");
    return order_sort(mesh, n, d_cell, d_death, d_order, d_n_live, d_scratch, o, (hipStream_t)stream);
}

// records[k][c][i] = 0 for k in [k0, K), slots i in [*n_live, n): blockIdx.y strides over the
// (k, c) rows, blocks wholly before the live count exit at once
__global__ void __launch_bounds__(256) records_clear_dead_kernel(int64_t n, const int32_t* __restrict__ n_live,
                                                                 int64_t k0, int64_t rows, double* __restrict__ rec,
                                                                 int64_t stride) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t nl = *n_live;
    if ((int64_t)(blockIdx.x + 1) * blockDim.x <= nl || i >= n || i < nl) return;
    for (int64_t r = blockIdx.y; r < rows; r += gridDim.y) rec[(k0 * 6 + r) * stride + i] = 0.0;
}

mops_status mops_records_clear_dead(int64_t n, const int32_t* d_n_live, int64_t k_begin, int64_t K,
                                    double* d_records, int64_t record_stride, void* stream) {
    if (n < 0 || k_begin < 0 || K < 0 || (n > 0 && (!d_n_live || !d_records)) || record_stride < n)
        return fail(MOPS_ERR_INVALID, "mops_records_clear_dead: invalid argument");
    if (n == 0 || k_begin >= K) return MOPS_OK;
    const int64_t rows = (K - k_begin) * 6;
    const dim3 grid((unsigned)((n + 255) / 256), (unsigned)(rows < 1024 ? rows : 1024));
    records_clear_dead_kernel<<<grid, 256, 0, (hipStream_t)stream>>>(n, d_n_live, k_begin, rows, d_records,
                                                                     record_stride);
    HIP_TRY(hipGetLastError());
    return MOPS_OK;
}

int64_t mops_traj_num_records(const mops_traj_cfg* cfg) {
    if (!cfg || cfg->record_t <= 0) return 0;
    return cfg->simulation_duration / cfg->record_t;
}

int64_t mops_traj_num_steps(const mops_traj_cfg* cfg) {
    if (!cfg || cfg->delta_t <= 0) return 0;
    return cfg->simulation_duration / cfg->delta_t;
}

mops_status mops_traj_advance(const mops_mesh* mesh, const mops_field* front, const mops_field* back,
                              const mops_traj_cfg* cfg, const mops_particles* p, int64_t step_begin,
                              int64_t step_end, double* d_records, int64_t record_stride, void* stream) {
    if (!mesh || !front || !cfg || !p) return fail(MOPS_ERR_INVALID, "mops_traj_advance: invalid inputs");
    if (cfg->delta_t <= 0 || cfg->record_t <= 0 || cfg->simulation_duration <= 0)
        return fail(MOPS_ERR_INVALID, "invalid trajectory settings");  // :666-669
    const int64_t K = mops_traj_num_records(cfg), n_steps = mops_traj_num_steps(cfg);
    if (K <= 0 || n_steps <= 0) return fail(MOPS_ERR_INVALID, "invalid integration steps");  // :709-712
    if (front->mesh != mesh || (back && back->mesh != mesh)) return fail(MOPS_ERR_INVALID, "field/mesh mismatch");
    if (p->n < 0 || record_stride < p->n) return fail(MOPS_ERR_INVALID, "record_stride < n");
    if (p->n == 0) return MOPS_OK;
    if (!p->d_x || !p->d_y || !p->d_z || !p->d_depth || !p->d_cell || !p->d_death_step || !d_records)
        return fail(MOPS_ERR_INVALID, "mops_traj_advance: null device pointer");
    step_begin = std::max<int64_t>(step_begin, 0);
    step_end = std::min<int64_t>(step_end, n_steps);
    if (step_begin >= step_end) return MOPS_OK;
    if (cfg->delta_t > INT32_MAX) return fail(MOPS_ERR_INVALID, "deltaT too large");
    TrajArgs a;
    a.cellrec = mesh->d_cellrec; a.cxyz = mesh->d_cxyz; a.vxyz = mesh->d_vxyz;
    a.C = (int)mesh->C; a.V = (int)mesh->V; a.L = mesh->L;
    a.f0 = dev::Field{front->d_zt, front->d_pr};
    a.f1 = back ? dev::Field{back->d_zt, back->d_pr} : a.f0;
    a.mono0 = front->d_mono;
    a.mono1 = back ? back->d_mono : front->d_mono;
    a.order = p->d_order;
    a.n_live = p->d_n_live;
    a.cpoly = mesh->d_cpoly;
    a.cnrm = mesh->d_cnrm;
    a.cedge = mesh->d_cedge;
    a.nbr = mesh->d_nbr;
    a.cpolyr = mesh->d_cpolyr;
    a.crank = mesh->d_cell_rank;
    a.px = p->d_x; a.py = p->d_y; a.pz = p->d_z; a.depth = p->d_depth; a.cell = p->d_cell; a.death = p->d_death_step;
    a.n = p->n;
    a.step_begin = step_begin; a.step_end = step_end; a.n_steps = n_steps;
    const int dt_sign = (cfg->direction == MOPS_FORWARD) ? 1 : -1;
    a.delta_t = dt_sign * (int)cfg->delta_t;
    a.dalpha = (double)a.delta_t / (double)cfg->simulation_duration;
    if (back) {
        a.rec_period = cfg->record_t / cfg->delta_t;  // record_interval (:1470)
    } else {
        a.rec_period = cfg->record_t / gcd64(cfg->record_t, cfg->delta_t);  // run_time % recordT == 0 (:994)
    }
    a.K = K;
    a.rec = d_records;
    a.rec_stride = record_stride;
    const bool euler = (cfg->method == MOPS_EULER);
    hipStream_t s = (hipStream_t)stream;
    a.coop_sel = nullptr;
    if ((euler ? MOPS_COOP_PE : MOPS_COOP_PR) && back && mesh->maxv == 7 && !p->d_order) {
        int* sel = nullptr;
        MOPS_TRY(coop_flag(mesh, s, &sel));
        coop_select_kernel<<<1, 256, 0, s>>>(p->n, p->d_cell, p->d_n_live, sel);
        a.coop_sel = sel;
    }
    a.handoff = (MOPS_RK4_HANDOFF && !euler && a.coop_sel) ? 1 : 0;
    switch (mesh->maxv) {
        case 7: launch_traj<7>(a, back != nullptr, euler, s); break;
#if !defined(MOPS_ONLY7)  // experiment builds: MAXV 7 instantiations only
        case 12: launch_traj<12>(a, back != nullptr, euler, s); break;
        default: launch_traj<20>(a, back != nullptr, euler, s); break;
#else
        default: return fail(MOPS_ERR_UNSUPPORTED, "experiment build: MAXV 7 only");
#endif
    }
    HIP_TRY(hipGetLastError());
    return MOPS_OK;
}

mops_status mops_traj_finalize(int64_t n, int64_t K, const double* d_seeds, const double* d_records,
                               int64_t stride, int32_t pathline, const int32_t* d_line, double* d_points,
                               double* d_vel, double* d_tmp, double* d_sal, double* d_last, void* stream) {
    if (n < 0 || K <= 0 || !d_seeds || !d_records || !d_points || stride < n)
        return fail(MOPS_ERR_INVALID, "mops_traj_finalize: invalid argument");
    if (n == 0) return MOPS_OK;
    hipStream_t s = (hipStream_t)stream;
    const unsigned nb = (unsigned)((n + kAsmSlots - 1) / kAsmSlots);
    if (K <= kAsmFull) {
        assemble_clean_kernel<<<nb, 256, 0, s>>>(n, (int)K, d_seeds, d_records, stride, pathline, d_line, d_points,
                                                 d_vel, d_tmp, d_sal, d_last);
    } else {
        assemble_kernel<<<nb, 256, 0, s>>>(n, K, d_seeds, d_records, stride, pathline, d_line, d_points, d_vel, d_tmp,
                                           d_sal);
        remove_nan_kernel<<<grid_for(n), kBlock, 0, s>>>(n, K + 1, nullptr, d_points, d_vel, d_tmp, d_sal, d_last,
                                                         d_line);
    }
    HIP_TRY(hipGetLastError());
    return MOPS_OK;
}

mops_status mops_traj_last_points(int64_t n, int64_t K, const double* d_seeds, const double* d_records,
                                  int64_t stride, const int32_t* d_line, double* d_last, void* stream) {
    if (n < 0 || K <= 0 || K > INT32_MAX || !d_seeds || !d_records || !d_last || stride < n)
        return fail(MOPS_ERR_INVALID, "mops_traj_last_points: invalid argument");
    if (n == 0) return MOPS_OK;
    last_point_kernel<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(n, (int)K, d_seeds, d_records,
                                                                                   stride, d_line, d_last);
    HIP_TRY(hipGetLastError());
    return MOPS_OK;
}

// error hook for the host writers in mops_io.cpp (not part of the public ABI)
__attribute__((visibility("hidden"))) mops_status mops_io_fail(mops_status st, const char* msg) {
    return fail(st, msg ? msg : "");
}

mops_status mops_lines_geo(int64_t n, int64_t P, const double* d_points, const double* d_velocity, double* d_geo,
                           void* stream) {
    if (n < 0 || P < 0 || ((n * P) > 0 && (!d_points || !d_geo)))
        return fail(MOPS_ERR_INVALID, "mops_lines_geo: invalid argument");
    const int64_t m = n * P;
    if (m == 0) return MOPS_OK;
    lines_geo_kernel<<<grid_for(m), kBlock, 0, (hipStream_t)stream>>>(m, d_points, d_velocity, d_geo);
    HIP_TRY(hipGetLastError());
    return MOPS_OK;
}

mops_status mops_remove_nan_lines(int64_t n, int64_t P, double* d_points, double* d_vel, double* d_tmp, double* d_sal,
                                  double* d_last, void* stream) {
    if (n < 0 || P <= 0 || !d_points) return fail(MOPS_ERR_INVALID, "mops_remove_nan_lines: invalid argument");
    if (n == 0) return MOPS_OK;
    remove_nan_kernel<<<grid_for(n), kBlock, 0, (hipStream_t)stream>>>(n, P, nullptr, d_points, d_vel, d_tmp, d_sal,
                                                                        d_last);
    HIP_TRY(hipGetLastError());
    return MOPS_OK;
}

mops_status mops_remove_nan_ragged(int64_t n, const int64_t* d_offsets, double* d_points, double* d_vel,
                                   double* d_tmp, double* d_sal, double* d_last, void* stream) {
    if (n < 0 || (n > 0 && (!d_offsets || !d_points)))
        return fail(MOPS_ERR_INVALID, "mops_remove_nan_ragged: invalid argument");
    if (n == 0) return MOPS_OK;
    remove_nan_kernel<<<grid_for(n), kBlock, 0, (hipStream_t)stream>>>(n, 0, d_offsets, d_points, d_vel, d_tmp, d_sal,
                                                                        d_last);
    HIP_TRY(hipGetLastError());
    return MOPS_OK;
}

const char* mops_build_id(void) { return MOPS_BUILD_ID; }

mops_status mops_run_trajectories(const mops_mesh* mesh, const mops_field* front, const mops_field* back,
                                  const mops_traj_cfg* cfg, int64_t n, const double* h_seeds, const float* h_depths,
                                  float depth, int32_t* h_cells, double* h_points, double* h_vel, double* h_tmp,
                                  double* h_sal, double* h_last, double* h_final_pos, float* h_final_depth,
                                  int32_t* h_death, void* stream) {
    if (!mesh || !front || !cfg) return fail(MOPS_ERR_INVALID, "invalid inputs");  // :659-662
    if (n <= 0) return MOPS_OK;                                                      // :663-665 (empty)
    if (!h_seeds || !h_points) return fail(MOPS_ERR_INVALID, "mops_run_trajectories: null host buffer");
    if (cfg->delta_t <= 0 || cfg->record_t <= 0 || cfg->simulation_duration <= 0)
        return fail(MOPS_ERR_INVALID, "invalid trajectory settings");
    const int64_t K = mops_traj_num_records(cfg), n_steps = mops_traj_num_steps(cfg);
    if (K <= 0 || n_steps <= 0) return fail(MOPS_ERR_INVALID, "invalid integration steps");
    hipStream_t s = (hipStream_t)stream;
    const int64_t P = K + 1;
    // SoA state + record slab, one allocation
    double *seeds = nullptr, *x = nullptr, *y = nullptr, *z = nullptr, *rec = nullptr;
    double *pts = nullptr, *vel = nullptr, *tmp = nullptr, *sal = nullptr, *last = nullptr;
    float* dep = nullptr;
    int *cells = nullptr, *death = nullptr, *order = nullptr;
    mops_status st = MOPS_OK;
    std::vector<double> hx((size_t)n), hy((size_t)n), hz((size_t)n);
    std::vector<float> hd((size_t)n);
    for (int64_t i = 0; i < n; ++i) {
        hx[i] = h_seeds[3 * i]; hy[i] = h_seeds[3 * i + 1]; hz[i] = h_seeds[3 * i + 2];
        hd[i] = h_depths ? h_depths[i] : depth;
    }
    auto cleanup = [&]() {
        (void)hipFree(seeds); (void)hipFree(x); (void)hipFree(y); (void)hipFree(z); (void)hipFree(rec); (void)hipFree(pts); (void)hipFree(vel);
        (void)hipFree(tmp); (void)hipFree(sal); (void)hipFree(last); (void)hipFree(dep); (void)hipFree(cells); (void)hipFree(death);
        (void)hipFree(order);
    };
    do {
        if ((st = upload(h_seeds, (size_t)(3 * n), &seeds, nullptr, s)) != MOPS_OK) break;
        if ((st = upload(hx.data(), (size_t)n, &x, nullptr, s)) != MOPS_OK) break;
        if ((st = upload(hy.data(), (size_t)n, &y, nullptr, s)) != MOPS_OK) break;
        if ((st = upload(hz.data(), (size_t)n, &z, nullptr, s)) != MOPS_OK) break;
        if ((st = upload(hd.data(), (size_t)n, &dep, nullptr, s)) != MOPS_OK) break;
        if ((st = dmalloc(&cells, (size_t)n, nullptr)) != MOPS_OK) break;
        if ((st = dmalloc(&death, (size_t)n, nullptr)) != MOPS_OK) break;
        if ((st = dmalloc(&rec, (size_t)(K * 6 * n), nullptr)) != MOPS_OK) break;
        if ((st = dmalloc(&pts, (size_t)(n * P * 3), nullptr)) != MOPS_OK) break;
        if ((st = dmalloc(&vel, (size_t)(n * P * 3), nullptr)) != MOPS_OK) break;
        if ((st = dmalloc(&tmp, (size_t)(n * P), nullptr)) != MOPS_OK) break;
        if ((st = dmalloc(&sal, (size_t)(n * P), nullptr)) != MOPS_OK) break;
        if ((st = dmalloc(&last, (size_t)(n * 3), nullptr)) != MOPS_OK) break;
        // (rec needs no clearing: the launch from step 0 writes every record slot)
        hipError_t e = hipMemsetAsync(death, 0xff, (size_t)n * sizeof(int), s);  // -1 = alive
        if (e != hipSuccess) { st = fail(MOPS_ERR_HIP, hipGetErrorString(e)); break; }
        // default_cell_id: entries < 0 are located (MPASOVisualizerKernels.cpp:683-690)
        std::vector<int32_t> hc((size_t)n, -1);
        bool need_locate = (h_cells == nullptr);
        if (h_cells) {
            for (int64_t i = 0; i < n; ++i) { hc[i] = h_cells[i]; if (hc[i] < 0) need_locate = true; }
        }
        if (need_locate) {
            int32_t* located = nullptr;
            if ((st = dmalloc(&located, (size_t)n, nullptr)) != MOPS_OK) break;
            st = mops_locate_cells(mesh, n, seeds, located, s);
            std::vector<int32_t> hl((size_t)n);
            if (st == MOPS_OK) {
                e = hipMemcpyAsync(hl.data(), located, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, s);
                if (e == hipSuccess) e = hipStreamSynchronize(s);
                if (e != hipSuccess) st = fail(MOPS_ERR_HIP, hipGetErrorString(e));
            }
            (void)hipFree(located);
            if (st != MOPS_OK) break;
            for (int64_t i = 0; i < n; ++i) if (hc[i] < 0) hc[i] = hl[i];
            if (h_cells) for (int64_t i = 0; i < n; ++i) h_cells[i] = hc[i];
        }
        e = hipMemcpyAsync(cells, hc.data(), (size_t)n * sizeof(int32_t), hipMemcpyHostToDevice, s);
        if (e != hipSuccess) { st = fail(MOPS_ERR_HIP, hipGetErrorString(e)); break; }
        if ((st = dmalloc(&order, (size_t)n, nullptr)) != MOPS_OK) break;
        if ((st = mops_order_particles(mesh, n, cells, order, stream)) != MOPS_OK) break;
        mops_particles prt{n, x, y, z, dep, cells, death, order, nullptr};
        if ((st = mops_traj_advance(mesh, front, back, cfg, &prt, 0, n_steps, rec, n, stream)) != MOPS_OK) break;
        if ((st = mops_traj_finalize(n, K, seeds, rec, n, back ? 1 : 0, nullptr, pts, vel, tmp, sal, last, stream)) !=
            MOPS_OK)
            break;
        e = hipMemcpyAsync(h_points, pts, (size_t)(n * P * 3) * sizeof(double), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && h_vel) e = hipMemcpyAsync(h_vel, vel, (size_t)(n * P * 3) * sizeof(double), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && h_tmp) e = hipMemcpyAsync(h_tmp, tmp, (size_t)(n * P) * sizeof(double), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && h_sal) e = hipMemcpyAsync(h_sal, sal, (size_t)(n * P) * sizeof(double), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && h_last) e = hipMemcpyAsync(h_last, last, (size_t)(n * 3) * sizeof(double), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && h_final_depth) e = hipMemcpyAsync(h_final_depth, dep, (size_t)n * sizeof(float), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && h_death) e = hipMemcpyAsync(h_death, death, (size_t)n * sizeof(int32_t), hipMemcpyDeviceToHost, s);
        if (e == hipSuccess && h_final_pos) {
            e = hipMemcpyAsync(hx.data(), x, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipMemcpyAsync(hy.data(), y, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipMemcpyAsync(hz.data(), z, (size_t)n * sizeof(double), hipMemcpyDeviceToHost, s);
        }
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        if (e != hipSuccess) { st = fail(MOPS_ERR_HIP, hipGetErrorString(e)); break; }
        if (h_final_pos)
            for (int64_t i = 0; i < n; ++i) {
                h_final_pos[3 * i] = hx[i]; h_final_pos[3 * i + 1] = hy[i]; h_final_pos[3 * i + 2] = hz[i];
            }
    } while (0);
    cleanup();
    return st;
}

}  // extern "C"
