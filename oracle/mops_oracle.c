/*
 * mops_oracle.c -- CPU restatement of the reference particle-trajectory path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker for the HIP
 * engine in mops_amd/csrc.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load it; the product path never does.
 *
 * It restates, function by function and in the same floating-point operation
 * order, the reference's TBB CPU path of YosefQiu/MOPS (snapshot 2026-05-15):
 *
 *   orc_streamline          src/CPU/TBB/Kernel/MPASOVisualizerKernels.cpp:653-1015
 *   orc_pathline            src/CPU/TBB/Kernel/MPASOVisualizerKernels.cpp:1017-1496
 *   is_in_mesh              src/CPU/TBB/Kernel/TBBKernel.h:21-54
 *   neighbors_idx           src/CPU/TBB/Kernel/TBBKernel.h:74-101
 *   rotate                  src/CPU/TBB/Kernel/TBBKernel.h:168-206
 *   wachspress/tri_area     src/Utils/Interpolation.hpp:95-110,137-165
 *   orc_gauss_elimination   src/Utils/Interpolation.hpp:174-217
 *   orc_center_velocity_rbf src/CPU/TBB/MPASOSolutionTBB.cpp:131-245 + Interpolation.hpp:167-340
 *   orc_cell_center_ztop    src/Core/MPASOSolution.cpp:535-618
 *   orc_cell_to_vertex      src/CPU/TBB/MPASOSolutionTBB.cpp:9-106, 270-366
 *   orc_center_velocity_zm  src/CPU/TBB/MPASOSolutionTBB.cpp:108-129 + GeoConverter.hpp:225-247
 *   orc_remove_nan          src/Common/TrajectoryCommon.h:57-129
 *   orc_knn                 src/Core/MPASOGrid.cpp:287-313 (nanoflann exact 1-NN)
 *
 * Parity status: the reference cannot be compiled in this image without
 * stand-ins (its headers include netcdf.h, tbb/ and ftk ndarray, none of
 * which exist here), so this restatement is pinned by the reference's own
 * test vectors (test/test_trajector.cpp:26-194, test/test_gaussian.cpp:9-27,
 * see tests/golden/) and by analytic invariants (tests/test_oracle.py).  The
 * full trajectory loop is therefore "partially pinned" (DESIGN.md §Parity).
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fno-fast-math -fopenmp).
 * Index convention: the oracle takes the reference's own storage form --
 * size_t (uint64) 1-based connectivity and AoS vec3 coordinates.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define MAX_VERTEX_NUM 20
#define MAX_LEVELS 100
#define MAX_NEIGH 21

typedef struct { double x, y, z; } v3;

static inline v3 mk(double x, double y, double z) { v3 r = {x, y, z}; return r; }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 mul(v3 a, double s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline v3 dvs(v3 a, double s) { return mk(a.x / s, a.y / s, a.z / s); }
/* cy::Vec3::Cross / Dot (cyVector.h:391-393); MOPS_LENGTH (BackendCompat.hpp:254) */
static inline v3 cross(v3 a, v3 p) { return mk(a.y * p.z - a.z * p.y, a.z * p.x - a.x * p.z, a.x * p.y - a.y * p.x); }
static inline double dot(v3 a, v3 p) { return a.x * p.x + a.y * p.y + a.z * p.z; }
static inline double len(v3 v) { return sqrt(v.x * v.x + v.y * v.y + v.z * v.z); }
static inline v3 ld(const double* a, int64_t i) { return mk(a[3 * i], a[3 * i + 1], a[3 * i + 2]); }
static inline double dmax(double a, double b) { return (a < b) ? b : a; }   /* std::max */
static inline double dmin(double a, double b) { return (b < a) ? b : a; }   /* std::min */
static inline double dclamp(double v, double lo, double hi) { return (v < lo) ? lo : (hi < v) ? hi : v; }

typedef struct {
    int64_t n_cells, n_vertices;
    int32_t max_edges, n_levels;          /* nVertLevels; the w grid has n_levels+1 */
    const uint64_t* n_edges_on_cell;      /* numberVertexOnCell_vec [C] */
    const uint64_t* vertices_on_cell;     /* [C*maxE], 1-based */
    const uint64_t* cells_on_cell;        /* [C*maxE], 1-based, 0 = none */
    const double* cell_coord;             /* [C*3] */
    const double* vertex_coord;           /* [V*3] */
} orc_mesh;

typedef struct {
    const double* vertex_ztop;            /* cellVertexZTop_vec   [V*L] */
    const double* vertex_vel;             /* cellVertexVelocity_vec [V*L*3] */
    const double* vertex_w;               /* cellVertexVertVelocity_vec [V*(L+1)] */
} orc_field;

typedef struct {
    int64_t delta_t, duration, record_t;  /* size_t deltaT, simulationDuration, recordT */
    int32_t backward;                     /* CalcDirection::kBackward */
    int32_t euler;                        /* CalcMethodType::kEuler (reference default) */
} orc_cfg;

/* ---------------- TBBKernel helpers ---------------- */

static int is_in_mesh(const orc_mesh* m, int cell, v3 p) {
    if (!isfinite(p.x) || !isfinite(p.y) || !isfinite(p.z)) return 0;
    uint64_t nv = m->n_edges_on_cell[cell];
    if (nv == 0) return 0;
    for (uint64_t k = 0; k < nv; ++k) {
        uint64_t a_idx = m->vertices_on_cell[(int64_t)cell * m->max_edges + k] - 1;
        uint64_t b_idx = m->vertices_on_cell[(int64_t)cell * m->max_edges + ((k + 1) % nv)] - 1;
        v3 a = ld(m->vertex_coord, (int64_t)a_idx), b = ld(m->vertex_coord, (int64_t)b_idx);
        v3 n = cross(a, b);
        if (dot(n, p) < 0.0) return 0;
    }
    return 1;
}

static void neighbors_idx(const orc_mesh* m, int cell, int nv, int* out) {
    if (nv > MAX_NEIGH) return;
    out[0] = cell;
    int copyN = nv;
    if (copyN > MAX_NEIGH - 1) copyN = MAX_NEIGH - 1;
    for (int k = 0; k < copyN; ++k)
        out[k] = (int)m->cells_on_cell[(int64_t)cell * m->max_edges + k] - 1;
    out[copyN] = cell;
    for (int k = copyN + 1; k < MAX_NEIGH; ++k) out[k] = -1;
}

static v3 rot_axis(v3 p, v3 v) {
    return mk(p.y * v.z - p.z * v.y, p.z * v.x - p.x * v.z, p.x * v.y - p.y * v.x);
}

static v3 rotate(v3 p, v3 axis, double theta) {
    const double c = cos(theta), s = sin(theta);
    const double al = len(axis);
    if (al <= 1e-12) return p;
    v3 u = mk(axis.x / al, axis.y / al, axis.z / al);
    v3 r;
    r.x = (c + u.x * u.x * (1.0 - c)) * p.x + (u.x * u.y * (1.0 - c) - u.z * s) * p.y + (u.x * u.z * (1.0 - c) + u.y * s) * p.z;
    r.y = (u.y * u.x * (1.0 - c) + u.z * s) * p.x + (c + u.y * u.y * (1.0 - c)) * p.y + (u.y * u.z * (1.0 - c) - u.x * s) * p.z;
    r.z = (u.z * u.x * (1.0 - c) - u.y * s) * p.x + (u.z * u.y * (1.0 - c) + u.x * s) * p.y + (c + u.z * u.z * (1.0 - c)) * p.z;
    return r;
}

static v3 advect_on_sphere(v3 pos, v3 vel, double dt) {
    const double rr = len(pos), sp = len(vel);
    if (rr < 1e-12 || sp < 1e-12) return pos;
    v3 axis = rot_axis(pos, vel);
    const double theta = (sp * dt) / rr;
    return rotate(pos, axis, theta);
}

/* Interpolator::triangle_area / CalcPolygonWachspress */
static double tri_area(v3 a, v3 b, v3 c) {
    v3 e1 = mk(b.x - a.x, b.y - a.y, b.z - a.z);
    v3 e2 = mk(c.x - a.x, c.y - a.y, c.z - a.z);
    v3 cp = mk(e1.y * e2.z - e1.z * e2.y, e1.z * e2.x - e1.x * e2.z, e1.x * e2.y - e1.y * e2.x);
    return sqrt(cp.x * cp.x + cp.y * cp.y + cp.z * cp.z) / 2.0;
}

static void wachspress(v3 p, const v3* poly, double* w, int N) {
    for (int i = 0; i < N; i++) w[i] = 0.0;
    double sum = 0.0, Ai, Aip1, B;
    Aip1 = tri_area(poly[N - 1], poly[0], p);
    for (int i = 0; i < N; i++) {
        Ai = Aip1;
        Aip1 = tri_area(poly[i], poly[(i + 1) % N], p);
        B = tri_area(poly[(i - 1 + N) % N], poly[i], poly[(i + 1) % N]);
        w[i] = B / (Ai * Aip1);
        sum += w[i];
    }
    double recp = 1.0 / sum;
    for (int i = 0; i < N; i++) w[i] *= recp;
}

/* Common front half of calc_velocity_at: guards, IsInMesh, weights. */
typedef struct { int nv; int64_t vid[MAX_VERTEX_NUM]; double w[MAX_VERTEX_NUM]; } stencil_t;

static int build_stencil(const orc_mesh* m, int cell, v3 pos, stencil_t* st) {
    const int L = m->n_levels;
    if (cell < 0 || L <= 1 || L > MAX_LEVELS) return 0;
    int nv = (int)m->n_edges_on_cell[cell];
    if (nv <= 0 || nv > MAX_VERTEX_NUM) return 0;
    if (!is_in_mesh(m, cell, pos)) return 0;
    v3 poly[MAX_VERTEX_NUM];
    for (int k = 0; k < nv; ++k) {
        uint64_t vid = m->vertices_on_cell[(int64_t)cell * m->max_edges + k] - 1;
        st->vid[k] = (int64_t)vid;
        poly[k] = ld(m->vertex_coord, (int64_t)vid);
    }
    st->nv = nv;
    wachspress(pos, poly, st->w, nv);
    return 1;
}

static int column(const orc_mesh* m, const stencil_t* st, const double* zt, double* z) {
    const int L = m->n_levels;
    for (int k = 0; k < L; ++k) {
        double acc = 0.0;
        for (int v = 0; v < st->nv; ++v) {
            const int vid = (int)st->vid[v];
            if (vid < 0 || vid >= m->n_vertices) return 0;
            acc += st->w[v] * zt[(int64_t)vid * L + k];
        }
        z[k] = acc;
    }
    for (int k = 1; k < L; ++k)
        if (z[k] > z[k - 1]) z[k] = z[k - 1] - 1e-9;
    return 1;
}

static v3 calc_vel(const stencil_t* st, int Lt, int layer, const double* vel) {
    v3 r = mk(0.0, 0.0, 0.0);
    for (int v = 0; v < st->nv; ++v) {
        const int64_t i = st->vid[v] * Lt + layer;
        r.x += st->w[v] * vel[3 * i];
        r.y += st->w[v] * vel[3 * i + 1];
        r.z += st->w[v] * vel[3 * i + 2];
    }
    return r;
}

static double calc_attr(const stencil_t* st, int Lt, int layer, const double* a) {
    double r = 0.0;
    for (int v = 0; v < st->nv; ++v) r += st->w[v] * a[st->vid[v] * Lt + layer];
    return r;
}

typedef struct { v3 h; double w; int ok; } vstate;

/* streamline calc_velocity_at (MPASOVisualizerKernels.cpp:740-872) */
static vstate vel_stream(const orc_mesh* m, const orc_field* f, v3 pos, int cell, double depth) {
    vstate bad = {{0, 0, 0}, 0.0, 0};
    stencil_t st;
    if (!build_stencil(m, cell, pos, &st)) return bad;
    const int L = m->n_levels;
    double z[MAX_LEVELS];
    if (!column(m, &st, f->vertex_ztop, z)) return bad;
    const double eps = 1e-8;
    int layer = -1;
    if (depth > z[0] + eps) layer = 1;
    else if (depth < z[L - 1] - eps) layer = L - 1;
    else {
        int lo = 1, hi = L - 1, ans = 1;
        while (lo <= hi) {
            const int mid = (lo + hi) >> 1;
            const double top = z[mid - 1], bot = z[mid];
            if (depth <= top + eps && depth >= bot - eps) { ans = mid; break; }
            if (depth > top + eps) hi = mid - 1; else lo = mid + 1;
        }
        if (ans < 1) ans = 1;
        if (ans > L - 1) ans = L - 1;
        layer = ans;
    }
    if (layer < 0) return bad;
    const double zdn = z[layer], zup = z[layer - 1];
    double x = depth;
    x = dmax(zdn, dmin(x, zup));
    const double den = zup - zdn;
    if (fabs(den) < 1e-12) return bad;
    const double t = (x - zdn) / den;
    v3 vdn = calc_vel(&st, L, layer, f->vertex_vel);
    v3 vup = calc_vel(&st, L, layer - 1, f->vertex_vel);
    if (len(vdn) < 1e-12 || len(vup) < 1e-12) return bad;
    v3 fv = add(mul(vup, t), mul(vdn, 1.0 - t));
    if (len(fv) < 1e-12) return bad;
    const int Lp1 = L + 1;
    int dn_if = layer, up_if = (layer > 0) ? (layer - 1) : 0;
    if (dn_if >= Lp1) dn_if = Lp1 - 1;
    if (up_if >= Lp1) up_if = Lp1 - 1;
    const double wdn = calc_attr(&st, Lp1, dn_if, f->vertex_w);
    const double wup = calc_attr(&st, Lp1, up_if, f->vertex_w);
    vstate r;
    r.h = fv; r.w = t * wup + (1.0 - t) * wdn; r.ok = 1;
    return r;
}

/* PathLine front/back bracket (MPASOVisualizerKernels.cpp:1182-1218).
 * Q4: the reference picks layer 0 above the surface and then reads z[-1]
 * (undefined behaviour).  The restatement uses layer 1 there (the StreamLine
 * rule, :793-794) -- a documented, deliberate deviation at a UB site. */
static int path_layer(const double* z, int L, double d) {
    const double eps = 1e-8;
    if (d > z[0] + eps) return 1;               /* reference: 0 (UB) */
    if (d < z[L - 1] - eps) return L - 1;
    for (int k = 1; k < L; ++k)
        if (d <= z[k - 1] + eps && d >= z[k] - eps) return k;
    return -1;
}

/* pathline calc_velocity_at (MPASOVisualizerKernels.cpp:1124-1327); the
 * attribute channel is not computed: FinalizeTrajectoryLinesWithAttrs never
 * reads it (Q9, TrajectoryCommon.h:176-185), so it is unobservable. */
static vstate vel_path(const orc_mesh* m, const orc_field* ff, const orc_field* fb, v3 pos, int cell,
                       double depth, double alpha) {
    vstate bad = {{0, 0, 0}, 0.0, 0};
    stencil_t st;
    if (!build_stencil(m, cell, pos, &st)) return bad;
    const int L = m->n_levels;
    double zf[MAX_LEVELS], zb[MAX_LEVELS];
    /* the reference computes both columns in one fused loop; the per-element
     * arithmetic is identical to two separate passes */
    if (!column(m, &st, ff->vertex_ztop, zf)) return bad;
    if (!column(m, &st, fb->vertex_ztop, zb)) return bad;
    const int lf = path_layer(zf, L, depth), lb = path_layer(zb, L, depth);
    if (lf < 0 || lb < 0) return bad;
    const double zfdn = zf[lf], zfup = zf[lf - 1], zbdn = zb[lb], zbup = zb[lb - 1];
    double xf = dmax(zfdn, dmin(depth, zfup));
    double denf = zfup - zfdn;
    if (fabs(denf) < 1e-12) return bad;
    double tf = (xf - zfdn) / denf;
    double xb = dmax(zbdn, dmin(depth, zbup));
    double denb = zbup - zbdn;
    if (fabs(denb) < 1e-12) return bad;
    double tb = (xb - zbdn) / denb;
    v3 vdnf = calc_vel(&st, L, lf, ff->vertex_vel), vupf = calc_vel(&st, L, lf - 1, ff->vertex_vel);
    v3 fvf = add(mul(vupf, tf), mul(vdnf, 1.0 - tf));
    v3 vdnb = calc_vel(&st, L, lb, fb->vertex_vel), vupb = calc_vel(&st, L, lb - 1, fb->vertex_vel);
    v3 fvb = add(mul(vupb, tb), mul(vdnb, 1.0 - tb));
    v3 h = add(mul(fvb, alpha), mul(fvf, 1.0 - alpha));
    const int Lp1 = L + 1;
    int dnf = lf, upf = (lf > 0) ? lf - 1 : 0, dnb = lb, upb = (lb > 0) ? lb - 1 : 0;
    if (dnf >= Lp1) dnf = Lp1 - 1;
    if (upf >= Lp1) upf = Lp1 - 1;
    if (dnb >= Lp1) dnb = Lp1 - 1;
    if (upb >= Lp1) upb = Lp1 - 1;
    double wdnf = calc_attr(&st, Lp1, dnf, ff->vertex_w), wupf = calc_attr(&st, Lp1, upf, ff->vertex_w);
    double wf = tf * wupf + (1.0 - tf) * wdnf;
    double wdnb = calc_attr(&st, Lp1, dnb, fb->vertex_w), wupb = calc_attr(&st, Lp1, upb, fb->vertex_w);
    double wb = tb * wupb + (1.0 - tb) * wdnb;
    vstate r;
    r.h = h; r.w = alpha * wb + (1.0 - alpha) * wf; r.ok = 1;
    return r;
}

/* Shared per-particle driver.  Outputs the reference's raw host buffers:
 * rec_pos/rec_vel [N*K*3] (caller zero-initialises, as vector<vec3>::resize
 * does), plus the final stable_points/effective_depths and, as a diagnostic,
 * the step at which a particle died (-1 = survived) and its last cell. */
static void run_particle(const orc_mesh* m, const orc_field* ff, const orc_field* fb, const orc_cfg* cfg,
                         int64_t pid, double* pts, float* depths, const int32_t* cell0,
                         double* rec_pos, double* rec_vel, int32_t* death, int32_t* last_cell) {
    const int pathline = (fb != NULL);
    const int64_t K = cfg->duration / cfg->record_t;
    const int n_steps = (int)(cfg->duration / cfg->delta_t);
    const int dt_sign = cfg->backward ? -1 : 1;
    const int delta_t = dt_sign * (int)cfg->delta_t;
    const int C = (int)m->n_cells;
    const int64_t base = pid * K;
    int run_time = 0, first_loop = 1, first_vel = 1;
    int64_t rec_idx = 0;
    int cell = -1;
    int neig[MAX_NEIGH];
    for (int i = 0; i < MAX_NEIGH; ++i) neig[i] = -1;
    if (death) death[pid] = -1;
    for (int step = 0; step < n_steps; ++step) {
        const double alpha = (double)step / (double)n_steps;
        if (pathline) run_time += delta_t; else run_time += abs(delta_t);
        v3 p = ld(pts, pid);
        const double depth = -1.0 * (double)depths[pid];
        if (first_loop) {
            first_loop = 0;
            cell = cell0[pid];
            if (cell < 0 || cell >= C) { if (death) death[pid] = step; goto out; }
            neighbors_idx(m, cell, (int)m->n_edges_on_cell[cell], neig);
            rec_pos[3 * base] = p.x; rec_pos[3 * base + 1] = p.y; rec_pos[3 * base + 2] = p.z;
        } else {
            if (cell < 0 || cell >= C) { if (death) death[pid] = step; goto out; }
            int nv = (int)m->n_edges_on_cell[cell];
            double best = DBL_MAX;
            for (int n = 0; n < nv + 1; ++n) {
                int cid = neig[n];
                if (cid < 0 || cid >= C) continue;
                const double l = len(sub(ld(m->cell_coord, cid), p));
                if (l < best) { best = l; cell = cid; }
            }
            neighbors_idx(m, cell, (int)m->n_edges_on_cell[cell], neig);
        }
        const v3 cur = p;
        const double r = len(cur);
        v3 rk4_next = cur, hvel = mk(0, 0, 0);
        double vvel = 0.0;
        if (cfg->euler) {
            vstate s = pathline ? vel_path(m, ff, fb, cur, cell, depth, alpha) : vel_stream(m, ff, cur, cell, depth);
            if (!s.ok) { if (death) death[pid] = step; goto out; }
            hvel = s.h; vvel = s.w;
        } else {
            const double dt = (double)delta_t;
            const double dal = pathline ? dt / (double)cfg->duration : 0.0;
            const double a1 = alpha;
            vstate s1 = pathline ? vel_path(m, ff, fb, cur, cell, depth, a1) : vel_stream(m, ff, cur, cell, depth);
            if (!s1.ok) { if (death) death[pid] = step; goto out; }
            v3 p2 = advect_on_sphere(cur, s1.h, dt * 0.5);
            const double a2 = dclamp(a1 + 0.5 * dal, 0.0, 1.0);
            vstate s2 = pathline ? vel_path(m, ff, fb, p2, cell, depth, a2) : vel_stream(m, ff, p2, cell, depth);
            if (!s2.ok) { if (death) death[pid] = step; goto out; }
            v3 p3 = advect_on_sphere(cur, s2.h, dt * 0.5);
            const double a3 = dclamp(a1 + 0.5 * dal, 0.0, 1.0);
            vstate s3 = pathline ? vel_path(m, ff, fb, p3, cell, depth, a3) : vel_stream(m, ff, p3, cell, depth);
            if (!s3.ok) { if (death) death[pid] = step; goto out; }
            v3 p4 = advect_on_sphere(cur, s3.h, dt);
            const double a4 = dclamp(a1 + dal, 0.0, 1.0);
            vstate s4 = pathline ? vel_path(m, ff, fb, p4, cell, depth, a4) : vel_stream(m, ff, p4, cell, depth);
            if (!s4.ok) { if (death) death[pid] = step; goto out; }
            hvel = dvs(add(add(add(s1.h, mul(s2.h, 2.0)), mul(s3.h, 2.0)), s4.h), 6.0);
            vvel = (s1.w + 2.0 * s2.w + 2.0 * s3.w + s4.w) / 6.0;
            v3 xt = add(cur, mul(hvel, dt));
            const double xl = len(xt);
            rk4_next = (xl > 1e-12) ? mul(dvs(xt, xl), r) : cur;
        }
        v3 np_;
        if (cfg->euler) {
            v3 axis = rot_axis(cur, hvel);
            const double speed = len(hvel);
            const double theta = (speed * delta_t) / dmax(1e-12, r);
            np_ = rotate(cur, axis, theta);
        } else {
            np_ = rk4_next;
        }
        const double old_depth = (double)depths[pid];
        double nd = old_depth - vvel * (double)delta_t;
        nd = dmax(0.0, nd);
        const double r_new = dmax(1.0, r + vvel * (double)delta_t);
        depths[pid] = (float)nd;
        const double nl = len(np_);
        if (nl > 1e-12) np_ = mul(dvs(np_, nl), r_new);
        if (first_vel) {
            first_vel = 0;
            rec_vel[3 * base] = hvel.x; rec_vel[3 * base + 1] = hvel.y; rec_vel[3 * base + 2] = hvel.z;
        }
        pts[3 * pid] = np_.x; pts[3 * pid + 1] = np_.y; pts[3 * pid + 2] = np_.z;
        int record;
        if (pathline) {
            const int interval = (int)(cfg->record_t / cfg->delta_t);
            record = (interval > 0 && ((step + 1) % interval) == 0);
        } else {
            record = (cfg->record_t > 0 && (run_time % (int)cfg->record_t) == 0);
        }
        if (record) {
            if (rec_idx < K) {
                const int64_t w = base + rec_idx;
                rec_pos[3 * w] = np_.x; rec_pos[3 * w + 1] = np_.y; rec_pos[3 * w + 2] = np_.z;
                rec_vel[3 * w] = hvel.x; rec_vel[3 * w + 1] = hvel.y; rec_vel[3 * w + 2] = hvel.z;
            }
            ++rec_idx;
        }
    }
out:
    if (last_cell) last_cell[pid] = cell;
}

static int cfg_ok(const orc_cfg* c) {
    if (c->delta_t <= 0 || c->record_t <= 0 || c->duration <= 0) return 0;
    if (c->duration / c->record_t <= 0 || c->duration / c->delta_t <= 0) return 0;
    return 1;
}

static void run_all(const orc_mesh* m, const orc_field* ff, const orc_field* fb, const orc_cfg* cfg, int64_t n,
                    double* pts, float* depths, const int32_t* cells, double* rp, double* rv, int32_t* death,
                    int32_t* last_cell, int n_threads) {
#ifdef _OPENMP
    if (n_threads > 0) {
#pragma omp parallel for schedule(dynamic, 16) num_threads(n_threads)
        for (int64_t i = 0; i < n; ++i) run_particle(m, ff, fb, cfg, i, pts, depths, cells, rp, rv, death, last_cell);
        return;
    }
#endif
    (void)n_threads;
    for (int64_t i = 0; i < n; ++i) run_particle(m, ff, fb, cfg, i, pts, depths, cells, rp, rv, death, last_cell);
}

/* Returns 0 on success, -1 on invalid settings (reference: Error() + empty result). */
int orc_streamline(const orc_mesh* m, const orc_field* f, const orc_cfg* cfg, int64_t n, double* pts,
                   float* depths, const int32_t* cells, double* rec_pos, double* rec_vel, int32_t* death,
                   int32_t* last_cell, int n_threads) {
    if (!m || !f || !cfg || !cfg_ok(cfg)) return -1;
    run_all(m, f, NULL, cfg, n, pts, depths, cells, rec_pos, rec_vel, death, last_cell, n_threads);
    return 0;
}

int orc_pathline(const orc_mesh* m, const orc_field* ff, const orc_field* fb, const orc_cfg* cfg, int64_t n,
                 double* pts, float* depths, const int32_t* cells, double* rec_pos, double* rec_vel,
                 int32_t* death, int32_t* last_cell, int n_threads) {
    if (!m || !ff || !fb || !cfg || !cfg_ok(cfg)) return -1;
    run_all(m, ff, fb, cfg, n, pts, depths, cells, rec_pos, rec_vel, death, last_cell, n_threads);
    return 0;
}

/* ---------------- output assembly (TrajectoryCommon.h) ---------------- */

/* RemoveNaNTrajectoriesAndReindex for ONE line of P points with velocity,
 * temperature and salinity already resized to P (TrajectoryCommon.h:88-90).
 * Lines are never empty here (the seed is always pushed), so no line is
 * dropped and the new id equals the index. */
void orc_remove_nan(int64_t P, double* points, double* vel, double* temp, double* sal, double* last_point) {
    int64_t k = 0;
    for (; k < P; ++k)
        if (!isfinite(points[3 * k]) || !isfinite(points[3 * k + 1]) || !isfinite(points[3 * k + 2])) break;
    if (k == 0) {
        double fp[3] = {points[0], points[1], points[2]};
        double ft = temp[0], fs = sal[0];
        for (int64_t j = 0; j < P; ++j) {
            points[3 * j] = fp[0]; points[3 * j + 1] = fp[1]; points[3 * j + 2] = fp[2];
            vel[3 * j] = vel[3 * j + 1] = vel[3 * j + 2] = 0.0;
            temp[j] = ft; sal[j] = fs;
        }
    } else if (k < P) {
        double lp[3] = {points[3 * (k - 1)], points[3 * (k - 1) + 1], points[3 * (k - 1) + 2]};
        double lt = temp[k - 1], ls = sal[k - 1];
        vel[3 * (k - 1)] = vel[3 * (k - 1) + 1] = vel[3 * (k - 1) + 2] = 0.0;
        for (int64_t j = k; j < P; ++j) {
            points[3 * j] = lp[0]; points[3 * j + 1] = lp[1]; points[3 * j + 2] = lp[2];
            vel[3 * j] = vel[3 * j + 1] = vel[3 * j + 2] = 0.0;
            temp[j] = lt; sal[j] = ls;
        }
    }
    last_point[0] = points[3 * (P - 1)];
    last_point[1] = points[3 * (P - 1) + 1];
    last_point[2] = points[3 * (P - 1) + 2];
}

/* FinalizeTrajectoryLines[WithAttrs] (TrajectoryCommon.h:131-190) for all N
 * lines: seeds [N*3], raw buffers [N*K*3] -> points/vel [N*(K+1)*3],
 * temp/sal [N*(K+1)], last [N*3].  with_attrs selects the PathLine variant
 * whose temperature/salinity are the velocity x/y (Q9). */
void orc_finalize(int64_t N, int64_t K, const double* seeds, const double* rec_pos, const double* rec_vel,
                  int with_attrs, double* points, double* vel, double* temp, double* sal, double* last) {
    const int64_t P = K + 1;
    for (int64_t i = 0; i < N; ++i) {
        double* pp = points + 3 * i * P;
        double* vv = vel + 3 * i * P;
        double* tt = temp + i * P;
        double* ss = sal + i * P;
        memcpy(pp, seeds + 3 * i, 3 * sizeof(double));
        memcpy(pp + 3, rec_pos + 3 * i * K, 3 * K * sizeof(double));
        memcpy(vv, rec_vel + 3 * i * K, 3 * K * sizeof(double));
        vv[3 * K] = vv[3 * K + 1] = vv[3 * K + 2] = 0.0;
        for (int64_t j = 0; j < K; ++j) {
            tt[j] = with_attrs ? rec_vel[3 * (i * K + j)] : 0.0;
            ss[j] = with_attrs ? rec_vel[3 * (i * K + j) + 1] : 0.0;
        }
        tt[K] = 0.0; ss[K] = 0.0;
        orc_remove_nan(P, pp, vv, tt, ss, last + 3 * i);
    }
}

/* ---------------- derived-field preprocessing ---------------- */

/* MPASOSolution::calcCellCenterZtop: bottom-up from bottomDepth, else
 * top-down from SSH, else surface 0. */
void orc_cell_center_ztop(int64_t C, int L, const double* thick, const double* bottom, const double* ssh,
                          double* ztop) {
    for (int64_t i = 0; i < C; ++i) {
        if (bottom) {
            double z = -bottom[i];
            for (int k = L - 1; k >= 0; --k) { z += thick[L * i + k]; ztop[i * L + k] = z; }
        } else if (ssh) {
            double z = ssh[i];
            ztop[i * L] = z;
            for (int j = 1; j < L; ++j) { z -= thick[L * i + j - 1]; ztop[i * L + j] = z; }
        } else {
            ztop[i * L] = 0.0;
            for (int j = 1; j < L; ++j) ztop[i * L + j] = ztop[i * L + j - 1] - thick[L * i + j - 1];
        }
    }
    for (int64_t i = 0; i < C * L; ++i) ztop[i] *= 1.0;
}

/* Interpolator::calcTriangleBarycentric (Interpolation.hpp:79-93) */
static void barycentric(v3 p, v3 a, v3 b, v3 c, double* u, double* v, double* w) {
    v3 v0 = sub(b, a), v1 = sub(c, a), v2 = sub(p, a);
    double d00 = dot(v0, v0), d01 = dot(v0, v1), d11 = dot(v1, v1), d20 = dot(v2, v0), d21 = dot(v2, v1);
    double den = d00 * d11 - d01 * d01;
    *v = (d11 * d20 - d01 * d21) / den;
    *w = (d00 * d21 - d01 * d20) / den;
    *u = 1.0 - *v - *w;
}

/* CalcCellVertexZtop / CalcCellCenterToVertex / CalcCellVertexVertVelocity /
 * CalcCellVertexVelocity (MPASOSolutionTBB.cpp): dim = 1 (scalar) or 3
 * (vec3), Lt = levels of the field, clamp_neg = CenterToVertex's
 * "out_val < 0 -> 0" (MPASOSolutionTBB.cpp:99-101). */
void orc_cell_to_vertex(int64_t C, int64_t V, int Lt, int dim, int clamp_neg, const uint64_t* cells_on_vertex,
                        const double* cell_coord, const double* vertex_coord, const double* src, double* dst) {
    for (int64_t vid = 0; vid < V; ++vid) {
        uint64_t ids[3];
        for (int t = 0; t < 3; ++t) ids[t] = cells_on_vertex[3 * vid + t] - 1;
        int boundary = 0;
        for (int t = 0; t < 3; ++t) if (ids[t] > (uint64_t)(C + 1)) boundary = 1;
        double u = 0, v = 0, w = 0;
        if (!boundary)
            barycentric(ld(vertex_coord, vid), ld(cell_coord, (int64_t)ids[0]), ld(cell_coord, (int64_t)ids[1]),
                        ld(cell_coord, (int64_t)ids[2]), &u, &v, &w);
        for (int k = 0; k < Lt; ++k) {
            for (int d = 0; d < dim; ++d) {
                double out = 0.0;
                if (!boundary) {
                    const double a0 = src[((int64_t)ids[0] * Lt + k) * dim + d];
                    const double a1 = src[((int64_t)ids[1] * Lt + k) * dim + d];
                    const double a2 = src[((int64_t)ids[2] * Lt + k) * dim + d];
                    out = u * a0 + v * a1 + w * a2;
                    if (clamp_neg && out < 0.0) out = 0.0;
                }
                dst[(vid * Lt + k) * dim + d] = out;
            }
        }
    }
}

/* CalcCellCenterVelocityByZM + GeoConverter::convertENUVelocityToXYZ (Uup = 0) */
void orc_center_velocity_zm(int64_t C, int L, const double* cell_coord, const double* zonal, const double* mer,
                            double* out) {
    for (int64_t c = 0; c < C; ++c) {
        v3 p = ld(cell_coord, c);
        for (int k = 0; k < L; ++k) {
            const double uz = zonal[c * L + k], um = mer[c * L + k], uu = 0.0;
            double* o = out + 3 * (c * L + k);
            if (p.x == 0.0 && p.y == 0.0) { o[0] = 0.0; o[1] = 0.0; o[2] = uu; continue; }
            const double Rxy = sqrt(p.x * p.x + p.y * p.y);
            const double Rxyz = sqrt(p.x * p.x + p.y * p.y + p.z * p.z);
            const double slon = p.y / Rxy, clon = p.x / Rxy, slat = p.z / Rxyz, clat = Rxy / Rxyz;
            o[0] = -slon * uz - slat * clon * um + clon * clat * uu;
            o[1] = clon * uz - slat * slon * um + slon * clat * uu;
            o[2] = clat * um + slat * uu;
        }
    }
}

/* ---------------- seed location ---------------- */

/* Exact Euclidean 1-NN over cellCoord (nanoflann L2_Simple_Adaptor: squared
 * distance accumulated in dimension order).  Ties resolve to the smallest
 * index (nanoflann's tie order depends on tree traversal -- a measure-zero
 * event for real seeds, documented in DESIGN.md). */
void orc_knn(int64_t C, const double* cell_coord, int64_t n, const double* pts, int32_t* out, int n_threads) {
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(n_threads > 0 ? n_threads : 1)
#endif
    for (int64_t i = 0; i < n; ++i) {
        double best = DBL_MAX;
        int64_t bi = -1;
        for (int64_t c = 0; c < C; ++c) {
            double d0 = pts[3 * i] - cell_coord[3 * c], d1 = pts[3 * i + 1] - cell_coord[3 * c + 1],
                   d2 = pts[3 * i + 2] - cell_coord[3 * c + 2];
            double d = 0.0;
            d += d0 * d0; d += d1 * d1; d += d2 * d2;
            if (d < best) { best = d; bi = c; }
        }
        out[i] = (int32_t)bi;
    }
}

/* ---------------- RBF cell-centre velocity from edge normals ---------------- */

/* Interpolator::evaluate_rbf (Interpolation.hpp:169-172) */
static double rbf_eval(double r2) { return 1.0 / sqrt(1.0 + r2); }

/* Interpolator::gauss_elimination_fixed on the fixed 8 x 8 storage (Interpolation.hpp:174-217) */
static void gauss8(double A[8][8], double b[8], int n, double x[8]) {
    int pivot[8];
    for (int i = 0; i < n; i++) pivot[i] = i;
    for (int j = 0; j < n - 1; ++j) {
        int maxRow = j;
        for (int i = j + 1; i < n; ++i)
            if (fabs(A[pivot[i]][j]) > fabs(A[pivot[maxRow]][j])) maxRow = i;
        int tmp = pivot[j]; pivot[j] = pivot[maxRow]; pivot[maxRow] = tmp;
        for (int i = j + 1; i < n; ++i) {
            double factor = A[pivot[i]][j] / A[pivot[j]][j];
            A[pivot[i]][j] = factor;
            for (int k = j + 1; k < n; ++k) A[pivot[i]][k] -= factor * A[pivot[j]][k];
            b[pivot[i]] -= factor * b[pivot[j]];
        }
    }
    x[n - 1] = b[pivot[n - 1]] / A[pivot[n - 1]][n - 1];
    for (int i = n - 2; i >= 0; --i) {
        double sum = 0.0;
        for (int j = i + 1; j < n; ++j) sum += A[pivot[i]][j] * x[j];
        x[i] = (b[pivot[i]] - sum) / A[pivot[i]][i];
    }
}

/* Interpolator::mpas_rbf_interp_func_3D_plane_vec_const_dir_comp_coeffs (Interpolation.hpp:234-340) */
static void rbf_coeffs(int n, double src[8][3], double unit[8][3], const double dst[3], double alpha,
                       double pb[2][3], double coef[8][3]) {
    double ps[8][2] = {{0}}, pu[8][2] = {{0}}, pd[2] = {0};
    for (int i = 0; i < n; ++i) {
        ps[i][0] = src[i][0] * pb[0][0] + src[i][1] * pb[0][1] + src[i][2] * pb[0][2];
        ps[i][1] = src[i][0] * pb[1][0] + src[i][1] * pb[1][1] + src[i][2] * pb[1][2];
        pu[i][0] = unit[i][0] * pb[0][0] + unit[i][1] * pb[0][1] + unit[i][2] * pb[0][2];
        pu[i][1] = unit[i][0] * pb[1][0] + unit[i][1] * pb[1][1] + unit[i][2] * pb[1][2];
    }
    for (int d = 0; d < 2; ++d) pd[d] = dst[0] * pb[d][0] + dst[1] * pb[d][1] + dst[2] * pb[d][2];
    double A[8][8] = {{0}}, rhs[8][2] = {{0}};
    for (int j = 0; j < n; ++j) {
        for (int i = j; i < n; ++i) {
            double r2 = 0.0;
            for (int d = 0; d < 2; ++d) { double diff = ps[i][d] - ps[j][d]; r2 += diff * diff; }
            r2 /= (alpha * alpha);
            double rv = rbf_eval(r2);
            double dp = pu[i][0] * pu[j][0] + pu[i][1] * pu[j][1];
            A[i][j] = rv * dp;
            A[j][i] = A[i][j];
        }
        /* the reference computes the destination distance, then evaluates the RBF at 1.0 (:294-302) */
        double rdst = 0.0;
        for (int d = 0; d < 2; ++d) { double diff = pd[d] - ps[j][d]; rdst += diff * diff; }
        rdst /= (alpha * alpha);
        (void)rdst;
        double rvd = rbf_eval(1.0);
        rhs[j][0] = rvd * pu[j][0];
        rhs[j][1] = rvd * pu[j][1];
    }
    double x1[8] = {0}, x2[8] = {0}, Ac[8][8], b[8];
    for (int i = 0; i < n; ++i) for (int j = 0; j < n; ++j) Ac[i][j] = A[i][j];
    for (int i = 0; i < n; ++i) b[i] = rhs[i][0];
    gauss8(Ac, b, n, x1);
    for (int i = 0; i < n; ++i) for (int j = 0; j < n; ++j) Ac[i][j] = A[i][j];
    for (int i = 0; i < n; ++i) b[i] = rhs[i][1];
    gauss8(Ac, b, n, x2);
    for (int i = 0; i < n; ++i)
        for (int d = 0; d < 3; ++d) coef[i][d] = pb[0][d] * x1[i] + pb[1][d] * x2[i];
}

/* TBBBackend::CalcCellCenterVelocity (MPASOSolutionTBB.cpp:131-245): the cell-centre xyz velocity
 * [C*L*3] from the edge-normal velocity [E*L] by the reference's 7-point plane RBF (alpha forced to
 * 1, pointCount = MAX_VERTEX_NUM = 7 whatever nEdgesOnCell is: absent edges enter as zero points with
 * zero unit vectors).  Connectivity is the reference's size_t 1-based form (0 = none); every cell
 * must have nEdgesOnCell <= 7 (the reference's arrays hold 7). */
void orc_center_velocity_rbf(int64_t C, int L, int maxE, const uint64_t* n_edges_on_cell,
                             const uint64_t* edges_on_cell, const uint64_t* cells_on_edge, const double* edge_coord,
                             const double* cell_coord, const double* normal_vel, double* out) {
    const int NV = 7;
    const uint64_t none = UINT64_MAX;
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
    for (int64_t c = 0; c < C; ++c) {
        v3 pos = ld(cell_coord, c);
        const uint64_t nv = n_edges_on_cell[c];
        uint64_t eid[7];
        for (uint64_t k = 0; k < nv && k < 7; ++k) eid[k] = edges_on_cell[c * maxE + k] - 1;
        for (uint64_t k = nv; k < 7; ++k) eid[k] = none;
        v3 up = dvs(pos, len(pos));
        v3 east = cross(mk(0.0, 0.0, 1.0), up);
        if (len(east) < 1e-6) east = cross(mk(0.0, 1.0, 0.0), up);
        east = dvs(east, len(east));
        v3 north = cross(up, east);
        double pb[2][3] = {{east.x, east.y, east.z}, {north.x, north.y, north.z}};
        double center[3] = {pos.x, pos.y, pos.z};
        for (int k = 0; k < L; ++k) {
            double ec[8][3] = {{0}}, uv[8][3] = {{0}}, nvel[8] = {0}, coef[8][3] = {{0}};
            for (int s = 0; s < NV; ++s) {
                const uint64_t e = eid[s];
                if (e == none) continue;
                v3 ep = ld(edge_coord, (int64_t)e);
                ec[s][0] = ep.x; ec[s][1] = ep.y; ec[s][2] = ep.z;
                uint64_t c0 = cells_on_edge[e * 2 + 0] - 1, c1 = cells_on_edge[e * 2 + 1] - 1;
                uint64_t lo = c0 < c1 ? c0 : c1, hi = c0 > c1 ? c0 : c1;
                v3 nrm;
                double l;
                if (hi > (uint64_t)C) {
                    nrm = sub(ep, ld(cell_coord, (int64_t)lo));
                    l = len(nrm);
                    if (l == 0.0) continue;
                    nrm = dvs(nrm, l);
                } else {
                    nrm = sub(ld(cell_coord, (int64_t)hi), ld(cell_coord, (int64_t)lo));
                    l = len(nrm);
                    if (l == 0.0) continue;
                    nrm = dvs(nrm, l);
                }
                nvel[s] = normal_vel[e * (uint64_t)L + (uint64_t)k];
                uv[s][0] = nrm.x; uv[s][1] = nrm.y; uv[s][2] = nrm.z;
            }
            rbf_coeffs(NV, ec, uv, center, 1.0, pb, coef);
            double xv = 0.0, yv = 0.0, zv = 0.0;
            for (int s = 0; s < NV; ++s) {
                xv += coef[s][0] * nvel[s];
                yv += coef[s][1] * nvel[s];
                zv += coef[s][2] * nvel[s];
            }
            double* o = out + 3 * (c * L + k);
            o[0] = xv; o[1] = yv; o[2] = zv;
        }
    }
}

/* Interpolator::gauss_elimination_fixed (partial pivoting via an index permutation) on its fixed
 * 8 x 8 storage -- the solver of the RBF reconstruction above; pinned by test/test_gaussian.cpp:9-27
 * (tests/golden/gauss_kat.json).  A is n x n row-major, n <= 8 (copied; not modified). */
void orc_gauss_elimination(double* A, double* b, int n, double* x) {
    double a8[8][8] = {{0}}, b8[8] = {0}, x8[8] = {0};
    if (n < 1 || n > 8) return;
    for (int i = 0; i < n; ++i) {
        for (int j = 0; j < n; ++j) a8[i][j] = A[i * n + j];
        b8[i] = b[i];
    }
    gauss8(a8, b8, n, x8);
    for (int i = 0; i < n; ++i) x[i] = x8[i];
}

int orc_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
