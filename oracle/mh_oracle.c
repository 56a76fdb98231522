/*
 * mh_oracle.c -- TEST INFRASTRUCTURE ONLY (see mh_oracle.h).
 *
 * A plain-C restatement of the reference's per-chain hot path, Kernel.cu:162-828, written to
 * reproduce its arithmetic exactly: every value the reference holds in a float is rounded to a
 * float here at the same point, every double stays a double, and sums are taken in the
 * reference's loop order. Build with -ffp-contract=off (no fused multiply-add anywhere).
 *
 * Math library contract (shared with the device; DESIGN.md "Numerics"):
 *   - sqrt/sqrtf/division: IEEE correctly rounded on both sides;
 *   - every transcendental -- atan2 in theta, cos/sin of focalRot, exp in Accept, log/sin/cos in
 *     Box-Muller -- is the project's own (metropolis-hastings-gpgpu_amd/csrc/mh_math.h, fdlibm's
 *     algorithms, within ~1 ulp), compiled here by gcc and on the device by hipcc from the same
 *     source out of correctly rounded operations only, so both return the same bits by
 *     construction (tests/test_gpu_math.py checks it exhaustively on the 32-bit domains). The
 *     oracle includes that header only: it links nothing else of the product;
 *   - the reference's float transcendentals (atan2f in phi, cosf in FocalPointCosts) are taken
 *     as the double function rounded once to float, which is what a correctly rounded float
 *     library returns except in ~2^-29 of cases.
 *
 * Defined semantics where the reference is ill-defined:
 *   - one proposer per chain and a full state copy each step (the reference races when
 *     blockDim.x > 1, Kernel.cu:798, and copies with a broken stride, :733-734);
 *   - a drawn index == nObjs (u == 1.0f with nObjs >= 33, :566-574) counts as frozen and is
 *     redrawn; all-frozen rooms are a validation error instead of an endless loop (:600-602);
 *   - the chain's result is its final current state plus that state's cost components.
 */
#define _GNU_SOURCE
#include "mh_oracle.h"
#include "../metropolis-hastings-gpgpu_amd/csrc/mh_math.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* Constants, Kernel.cu:31-39. PI is 3.1416, not M_PI. */
#define ORC_PI (3.1416)
#define ORC_BETA (2.0)
#define ORC_S_SIGMA_T (15.0 / 90.0 * ORC_PI)

static __thread char g_err[256];

const char* orc_last_error(void) { return g_err; }

static int fail(const char* msg, long a) {
    snprintf(g_err, sizeof g_err, msg, a);
    return -1;
}

/* ------------------------------------------------------------------------------------------
 * RNG: rocRAND philox4x32_10_engine (rocrand_philox4x32_10.h), restated.
 * key = seed (lo, hi); counter = (0, 0, subsequence lo, subsequence hi); each block of four
 * outputs is ten Random123 Philox rounds of the counter; the counter then increments.
 * ---------------------------------------------------------------------------------------- */
#define PHILOX_M0 0xD2511F53u
#define PHILOX_M1 0xCD9E8D57u
#define PHILOX_W0 0x9E3779B9u
#define PHILOX_W1 0xBB67AE85u

void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int round = 0; round < 10; ++round) {
        uint64_t p0 = (uint64_t)PHILOX_M0 * c0;
        uint64_t p1 = (uint64_t)PHILOX_M1 * c2;
        uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        uint32_t n1 = (uint32_t)p1;
        uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        uint32_t n3 = (uint32_t)p0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        k0 += PHILOX_W0;
        k1 += PHILOX_W1;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

static void rng_refill(orc_rng* r) { orc_philox4x32_10(r->counter, r->key, r->result); }

static void rng_bump(orc_rng* r) {
    if (++r->counter[0] != 0) return;
    if (++r->counter[1] != 0) return;
    if (++r->counter[2] != 0) return;
    ++r->counter[3];
}

void orc_rng_init(orc_rng* r, uint64_t seed, uint64_t subsequence) {
    memset(r, 0, sizeof *r);
    r->key[0] = (uint32_t)seed;
    r->key[1] = (uint32_t)(seed >> 32);
    r->counter[2] = (uint32_t)subsequence;
    r->counter[3] = (uint32_t)(subsequence >> 32);
    rng_refill(r);
}

/* ------------------------------------------------------------------------------------------
 * cuRAND XORWOW (curandStateXORWOW_t; Kernel.cu:19 includes curand_kernel.h and :159 seeds
 * thread tid with curand_init(seed + tid, tid, 0)). cuRAND is not in this image; its published
 * algorithm is restated here: Marsaglia's xorwow (five xorshift words plus a Weyl sequence
 * d += 362437, output d + x4), seeded by scrambling the two 32-bit halves of the seed, with
 * subsequences 2^67 draws apart. The jump is computed here independently, as powers of the
 * 160 x 160 GF(2) transition matrix (the Weyl word needs no jump: 362437 * 2^67 = 0 mod 2^32).
 * ---------------------------------------------------------------------------------------- */
static void xw_step(uint32_t x[5]) {
    const uint32_t t = x[0] ^ (x[0] >> 2);
    x[0] = x[1];
    x[1] = x[2];
    x[2] = x[3];
    x[3] = x[4];
    x[4] = (x[4] ^ (x[4] << 4)) ^ (t ^ (t << 1));
}

/* Column k of a matrix is the image of basis vector e_k (word k / 32, bit k % 32). */
typedef struct { uint32_t col[160][5]; } xw_mat;

static void xw_apply(const xw_mat* m, const uint32_t v[5], uint32_t out[5]) {
    uint32_t o[5] = {0, 0, 0, 0, 0};
    for (int k = 0; k < 160; ++k)
        if ((v[k >> 5] >> (k & 31)) & 1u)
            for (int w = 0; w < 5; ++w) o[w] ^= m->col[k][w];
    memcpy(out, o, sizeof o);
}

static void xw_mul(const xw_mat* a, const xw_mat* b, xw_mat* out) { /* out = a * b */
    for (int k = 0; k < 160; ++k) xw_apply(a, b->col[k], out->col[k]);
}

static xw_mat g_xw_seq[64]; /* g_xw_seq[j] = A^(2^(67 + j)) */
static pthread_once_t g_xw_once = PTHREAD_ONCE_INIT;

static void xw_build_tables(void) {
    xw_mat* m = malloc(sizeof *m);
    xw_mat* t = malloc(sizeof *t);
    for (int k = 0; k < 160; ++k) {
        uint32_t e[5] = {0, 0, 0, 0, 0};
        e[k >> 5] = 1u << (k & 31);
        xw_step(e);
        memcpy(m->col[k], e, sizeof e);
    }
    for (int i = 0; i < 67; ++i) { /* A^(2^67) */
        xw_mul(m, m, t);
        memcpy(m, t, sizeof *m);
    }
    g_xw_seq[0] = *m;
    for (int j = 1; j < 64; ++j) xw_mul(&g_xw_seq[j - 1], &g_xw_seq[j - 1], &g_xw_seq[j]);
    free(m);
    free(t);
}

void orc_rng_init_xorwow(orc_rng* r, uint64_t seed, uint64_t subsequence, int kind) {
    memset(r, 0, sizeof *r);
    r->kind = kind;
    uint32_t s0, s1, t0, t1;
    if (kind == ORC_XORWOW_ROCRAND) { /* rocrand_xorwow.h xorwow_engine(seed, subsequence, 0) */
        s0 = (uint32_t)seed ^ 0x2c7f967fu;
        s1 = (uint32_t)(seed >> 32) ^ 0xa03697cbu;
        t0 = 1228688033u * s0;
        t1 = 2073658381u * s1;
    } else { /* cuRAND _curand_init_scratch */
        s0 = (uint32_t)seed ^ 0xaad26b49u;
        s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
        t0 = 1099087573u * s0;
        t1 = 2591861531u * s1;
    }
    uint32_t* x = r->xw + 1;
    r->xw[0] = 6615241u + t1 + t0;
    x[0] = 123456789u + t0;
    x[1] = 362436069u ^ t0;
    x[2] = 521288629u + t1;
    x[3] = 88675123u ^ t1;
    x[4] = 5783321u + t0;
    pthread_once(&g_xw_once, xw_build_tables);
    for (int j = 0; j < 64; ++j)
        if ((subsequence >> j) & 1u) xw_apply(&g_xw_seq[j], x, x);
}

static uint32_t xw_next(orc_rng* r) {
    xw_step(r->xw + 1);
    r->xw[0] += 362437u;
    return r->xw[0] + r->xw[5];
}

/* curand_uniform: x * 2^-32 + 2^-33 in float (Kernel.cu:569,710). */
static float xw_uniform(orc_rng* r) {
    float v = (float)xw_next(r);
    float scaled = v * 0x1p-32f;
    return scaled + 0x1p-33f;
}

/* curand_normal -> _curand_box_muller: u = x 2^-32 + 2^-33, v = fma(y, 2^-32 2pi_f, half of
 * it), s = sqrtf(-2 logf(u)), (sinf(v) s, cosf(v) s); sine branch first, cosine cached. The
 * float transcendentals are the double functions rounded once (see DESIGN.md "RNG modes"). */
static float xw_normal(orc_rng* r) {
    if (r->bm_has) {
        r->bm_has = 0;
        return r->bm_val;
    }
    const uint32_t a = xw_next(r), b = xw_next(r);
    const float k2pi = 0x1p-32f * 6.2831855f;
    const float u = (float)a * 0x1p-32f + 0x1p-33f;
    const float v = fmaf((float)b, k2pi, k2pi * 0.5f);
    const float lg = (float)mh_log((double)u);
    const float s = sqrtf(-2.0f * lg);
    double snd, csd;
    mh_sincos_medium((double)v, &snd, &csd);  /* (v <= 2 pi) */
    const float sn = (float)snd, cs = (float)csd;
    r->bm_val = cs * s;
    r->bm_has = 1;
    return sn * s;
}

uint32_t orc_rng_next(orc_rng* r) {
    if (r->kind) return xw_next(r);
    uint32_t v = r->result[r->substate];
    if (++r->substate == 4) {
        r->substate = 0;
        rng_bump(r);
        rng_refill(r);
    }
    return v;
}

/* rocrand_uniform (rocrand_uniform.h uniform_distribution): (0, 1], float arithmetic. Plays
 * the role of curand_uniform at Kernel.cu:569,710. */
float orc_rng_uniform(orc_rng* r) {
    if (r->kind) return xw_uniform(r);
    const float inv = 2.3283064e-10f;
    float v = (float)orc_rng_next(r);
    float scaled = v * inv;
    return inv + scaled;
}

/* Normal draw standing in for curand_normal (Kernel.cu:605,608,641): Box-Muller on two
 * uniforms in (0,1) evaluated in double and rounded to float; the sine branch is returned
 * first and the cosine branch is cached for the next call, as cuRAND's Box-Muller does. */
float orc_rng_normal(orc_rng* r) {
    if (r->kind) return xw_normal(r);
    if (r->bm_has) {
        r->bm_has = 0;
        return r->bm_val;
    }
    uint32_t a = orc_rng_next(r);
    uint32_t b = orc_rng_next(r);
    double u1 = (double)a * 0x1p-32 + 0x1p-33;
    double u2 = (double)b * 0x1p-32 + 0x1p-33;
    double rad = sqrt(-2.0 * mh_log(u1));
    double ang = 6.283185307179586 * u2;
    double sn, cs;
    mh_sincos_medium(ang, &sn, &cs);  /* (ang < 2 pi) */
    r->bm_val = (float)(rad * cs);
    r->bm_has = 1;
    return (float)(rad * sn);
}

/* rocrand_init(seed, subsequence, offset) for Philox4x32-10. */
void orc_rng_init_offset(orc_rng* r, uint64_t seed, uint64_t subsequence, uint64_t offset) {
    orc_rng_init(r, seed, subsequence);
    r->counter[0] = (uint32_t)(offset >> 2);
    r->counter[1] = (uint32_t)(offset >> 34);
    r->substate = (uint32_t)(offset & 3);
    rng_refill(r);
}

void orc_philox_stream(uint64_t seed, uint64_t subsequence, uint32_t* out, int n) {
    orc_rng r;
    orc_rng_init(&r, seed, subsequence);
    for (int i = 0; i < n; ++i) out[i] = orc_rng_next(&r);
}

/* ------------------------------------------------------------------------------------------
 * Geometry helpers.
 * ---------------------------------------------------------------------------------------- */
typedef struct { double x, y; } dvec2;

/* Kernel.cu:162-167: the difference is taken in float, the root in double. */
static double distance_f(float xi, float yi, float xj, float yj) {
    float fx = xi - xj;
    float fy = yi - yj;
    double dx = fx, dy = fy;
    double sq = dx * dx;
    sq = sq + dy * dy;
    return sqrt(sq);
}

/* Kernel.cu:170-182: bearing of i->j relative to ti, wrapped to [0, 2*PI) with PI = 3.1416. */
static double theta_f(float xi, float yi, float xj, float yj, float ti) {
    double dx = (double)(float)(xi - xj);
    double dy = (double)(float)(yi - yj);
    double tp = mh_atan2(dy, dx);
    if (tp < 0) tp = 2 * ORC_PI + tp;
    double t = tp - (double)ti;
    return (t < 0) ? 2 * ORC_PI + t : t;
}

/* float atan2 / cos as the double function rounded once (see header comment). */
static float atan2_f32(float y, float x) { return mh_atan2_f32(y, x); }
static float cos_f32(float x) { return mh_cos_f32(x); }

/* Kernel.cu:185-188: atan2 of float differences (float result), minus tj in float, plus
 * PI/2 in double, rounded to float on return. */
static float phi_f(float xi, float yi, float xj, float yj, float tj) {
    float a = atan2_f32(yi - yj, xi - xj);
    float b = a - tj;
    return (float)((double)b + ORC_PI / 2.0);
}

/* Kernel.cu:366-382 minValue: AABB minimum of the four consecutive vertices starting at
 * `start`, translated by (tx, ty). The first x candidate keeps the UNtranslated vertex
 * (Kernel.cu:371); y is translated throughout. */
static dvec2 aabb_min(const vertex* v, int start, float tx, float ty) {
    dvec2 m = {DBL_MAX, DBL_MAX};
    const vertex* q = v + start;
    m.x = (m.x > q[0].x + tx) ? q[0].x : m.x;
    for (int k = 1; k < 4; ++k) m.x = (m.x > q[k].x + tx) ? q[k].x + tx : m.x;
    for (int k = 0; k < 4; ++k) m.y = (m.y > q[k].y + ty) ? q[k].y + ty : m.y;
    return m;
}

/* Kernel.cu:384-401 maxValue: the translated maximum. */
static dvec2 aabb_max(const vertex* v, int start, float tx, float ty) {
    dvec2 m = {-DBL_MAX, -DBL_MAX};
    const vertex* q = v + start;
    for (int k = 0; k < 4; ++k) m.x = (m.x < q[k].x + tx) ? q[k].x + tx : m.x;
    for (int k = 0; k < 4; ++k) m.y = (m.y < q[k].y + ty) ? q[k].y + ty : m.y;
    return m;
}

/* Kernel.cu:321-340: overlap area of two AABBs; the double corners pass through fmaxf/fminf,
 * i.e. are rounded to float (so +-DBL_MAX becomes +-inf). */
static float overlap_area(dvec2 amin, dvec2 amax, dvec2 bmin, dvec2 bmax) {
    float x5 = fmaxf((float)amin.x, (float)bmin.x);
    float y5 = fmaxf((float)amin.y, (float)bmin.y);
    float x6 = fminf((float)amax.x, (float)bmax.x);
    float y6 = fminf((float)amax.y, (float)bmax.y);
    if (x5 >= x6 || y5 >= y6) return 0.0f;
    return (x6 - x5) * (y6 - y5);
}

/* Kernel.cu:343-364: the complement of the room AABB as four rectangles (min, max). */
static void complement_rects(dvec2 rmin, dvec2 rmax, dvec2 cmin[4], dvec2 cmax[4]) {
    cmin[0] = (dvec2){-DBL_MAX, -DBL_MAX}; cmax[0] = (dvec2){DBL_MAX, rmin.y};
    cmin[1] = (dvec2){-DBL_MAX, rmin.y};   cmax[1] = (dvec2){rmin.x, rmax.y};
    cmin[2] = (dvec2){-DBL_MAX, rmax.y};   cmax[2] = (dvec2){DBL_MAX, DBL_MAX};
    cmin[3] = (dvec2){rmax.x, rmin.y};     cmax[3] = (dvec2){DBL_MAX, rmax.y};
}

/* ------------------------------------------------------------------------------------------
 * Cost terms, Kernel.cu:191-514.
 * ---------------------------------------------------------------------------------------- */

/* Kernel.cu:191-207. Accumulators are floats updated through double temporaries. */
double orc_visual_balance(const orc_room* room, const positionAndRotation* cfg) {
    const Surface* s = room->srf;
    float nx = 0, ny = 0, denom = 0;
    for (int i = 0; i < s->nObjs; ++i) {
        float area = (float)(cfg[i].length * cfg[i].width);
        nx = (float)((double)nx + (double)area * cfg[i].x);
        ny = (float)((double)ny + (double)area * cfg[i].y);
        denom = denom + area;
    }
    return -1.0 * distance_f(nx / denom, ny / denom, (float)(s->centroidX / 2),
                             (float)(s->centroidY / 2));
}

/* Kernel.cu:210-233. */
double orc_pairwise(const orc_room* room, const positionAndRotation* cfg) {
    double acc = 0;
    for (int i = 0; i < room->srf->nRelationships; ++i) {
        const relationshipStruct* r = &room->rs[i];
        const positionAndRotation* a = &cfg[r->SourceIndex];
        const positionAndRotation* b = &cfg[r->TargetIndex];
        double d = distance_f((float)a->x, (float)a->y, (float)b->x, (float)b->y);
        if (d < r->TargetRange.targetRangeStart) {
            double f = d / r->TargetRange.targetRangeStart;
            acc -= f * f;
        } else if (d > r->TargetRange.targetRangeEnd) {
            double f = r->TargetRange.targetRangeEnd / d;
            acc -= f * f;
        }
    }
    return acc;
}

/* Kernel.cu:236-263, including the wrap branch's fmodf and the `min < d || d < max`
 * condition of the plain branch exactly as written. */
double orc_pairwise_angle(const orc_room* room, const positionAndRotation* cfg) {
    double acc = 0;
    for (int i = 0; i < room->srf->nRelationships; ++i) {
        const relationshipAngleStruct* r = &room->ra[i];
        const positionAndRotation* a = &cfg[r->SourceIndex];
        const positionAndRotation* b = &cfg[r->TargetIndex];
        double d = theta_f((float)a->x, (float)a->y, (float)b->x, (float)b->y, (float)b->rotY);
        double lo = r->angleMin, hi = r->angleMax;
        if (lo > hi) {
            double norm = (2 * ORC_PI - (hi + (2 * ORC_PI - lo))) / 2.0;
            float wrapped = fmodf((float)(lo + d), (float)(2 * ORC_PI));
            if ((double)wrapped > hi) acc -= fmin(fabs(d - lo), fabs(d - hi)) / norm;
        } else if (lo < d || d < hi) {
            double norm = (2 * ORC_PI - (hi - lo)) / 2.0;
            acc -= fmin(fabs(d - lo), fabs(d - hi)) / norm;
        }
    }
    return acc;
}

/* Kernel.cu:266-281. */
double orc_focal_point(const orc_room* room, const positionAndRotation* cfg) {
    const Surface* s = room->srf;
    double acc = 0;
    for (int i = 0; i < s->nObjs; ++i) {
        float p = phi_f((float)s->focalX, (float)s->focalY, (float)cfg[i].x, (float)cfg[i].y,
                        (float)cfg[i].rotY);
        acc -= (double)cos_f32(p);
    }
    return acc;
}

/* Kernel.cu:283-318. Reflect object i across the focal axis; score the best-matching j. */
float orc_symmetry(const orc_room* room, const positionAndRotation* cfg) {
    const Surface* s = room->srf;
    const int n = s->nObjs;
    float acc = 0;
    for (int i = 0; i < n; ++i) {
        float best = 0;
        float ux = (float)mh_cos(s->focalRot);
        float uy = (float)mh_sin(s->focalRot);
        double along_f = s->focalX * ux;
        along_f = along_f + s->focalY * uy;
        double along_i = cfg[i].x * ux;
        along_i = along_i + cfg[i].y * uy;
        float sd = (float)(2 * (along_f - along_i));
        float rx = (float)(cfg[i].x + (double)(sd * ux));
        float ry = (float)(cfg[i].y + (double)(sd * uy));
        float rrot = (float)(2 * s->focalRot - cfg[i].rotY);
        if (rrot < -ORC_PI) rrot = (float)((double)rrot + 2 * ORC_PI);
        for (int j = 0; j < n; ++j) {
            float dp = (float)distance_f((float)cfg[j].x, (float)cfg[j].y, rx, ry);
            float dt = (float)(cfg[j].rotY - (double)rrot);
            if (dt > ORC_PI) dt = (float)((double)dt - 2 * ORC_PI);
            float head = 5.0f - sqrtf(dp);
            float val = (float)((double)head - 0.4 * (double)fabsf(dt));
            best = fmaxf(best, val);
        }
        acc = acc - best;
    }
    return acc;
}

/* Kernel.cu:404-434: every clearance (at its source object) against every object's
 * off-limits rectangle, the source object included; float sum in i-major order. */
float orc_clearance(const orc_room* room, const positionAndRotation* cfg) {
    const Surface* s = room->srf;
    float err = 0.0f;
    for (int i = 0; i < s->nClearances; ++i) {
        const rectangle* c = &room->clearances[i];
        const positionAndRotation* src = &cfg[c->SourceIndex];
        for (int j = 0; j < s->nObjs; ++j) {
            dvec2 amin = aabb_min(room->vertices, c->point1Index, (float)src->x, (float)src->y);
            dvec2 amax = aabb_max(room->vertices, c->point1Index, (float)src->x, (float)src->y);
            int o = room->offlimits[j].point1Index;
            dvec2 bmin = aabb_min(room->vertices, o, (float)cfg[j].x, (float)cfg[j].y);
            dvec2 bmax = aabb_max(room->vertices, o, (float)cfg[j].x, (float)cfg[j].y);
            err -= overlap_area(amin, amax, bmin, bmax);
        }
    }
    return err;
}

/* Kernel.cu:437-483. Clearance i is translated by cfg[i] (not its source, :456). */
float orc_surface_area(const orc_room* room, const positionAndRotation* cfg) {
    const Surface* s = room->srf;
    dvec2 rmin = aabb_min(room->surfaceRectangle, 0, 0, 0);
    dvec2 rmax = aabb_max(room->surfaceRectangle, 0, 0, 0);
    dvec2 cmin[4], cmax[4];
    complement_rects(rmin, rmax, cmin, cmax);
    float err = 0.0f;
    for (int i = 0; i < s->nClearances; ++i) {
        int p = room->clearances[i].point1Index;
        dvec2 amin = aabb_min(room->vertices, p, (float)cfg[i].x, (float)cfg[i].y);
        dvec2 amax = aabb_max(room->vertices, p, (float)cfg[i].x, (float)cfg[i].y);
        for (int k = 0; k < 4; ++k) err -= overlap_area(amin, amax, cmin[k], cmax[k]);
    }
    for (int j = 0; j < s->nObjs; ++j) {
        int p = room->offlimits[j].point1Index;
        dvec2 amin = aabb_min(room->vertices, p, (float)cfg[j].x, (float)cfg[j].y);
        dvec2 amax = aabb_max(room->vertices, p, (float)cfg[j].x, (float)cfg[j].y);
        for (int k = 0; k < 4; ++k) err -= overlap_area(amin, amax, cmin[k], cmax[k]);
    }
    return err;
}

/* Kernel.cu:485-514: off-limits overlap over unordered pairs i < j. */
float orc_off_limits(const orc_room* room, const positionAndRotation* cfg) {
    const Surface* s = room->srf;
    float err = 0.0f;
    for (int i = 0; i < s->nObjs; ++i) {
        for (int j = i + 1; j < s->nObjs; ++j) {
            int pi = room->offlimits[i].point1Index, pj = room->offlimits[j].point1Index;
            dvec2 amin = aabb_min(room->vertices, pi, (float)cfg[i].x, (float)cfg[i].y);
            dvec2 amax = aabb_max(room->vertices, pi, (float)cfg[i].x, (float)cfg[i].y);
            dvec2 bmin = aabb_min(room->vertices, pj, (float)cfg[j].x, (float)cfg[j].y);
            dvec2 bmax = aabb_max(room->vertices, pj, (float)cfg[j].x, (float)cfg[j].y);
            err -= overlap_area(amin, amax, bmin, bmax);
        }
    }
    return err;
}

/* Kernel.cu:516-550. PairWise is the PRODUCT of the distance and angle terms (:518); the
 * total leaves OffLimits out (:547) and is summed in float in the reference's order. */
/* OffLimitsCosts in every step's Costs() (1, the reference's loop, :516-550 via :800) or only
 * for the configurations a chain outputs (0). OffLimits never enters totalCosts (:547), so no
 * accept decision depends on it, and a chain's output costs are Costs() of its output
 * configuration either way: 0 gives the same outputs bit for bit in about half the time at
 * N = 64 (the parity tests use it; the CPU baseline keeps the reference's loop). */
static int g_step_offlimits = 1;

void orc_set_step_offlimits(int on) { g_step_offlimits = on != 0; }

static void costs_ex(const orc_room* room, const positionAndRotation* cfg, resultCosts* out,
                     int with_ol);

void orc_costs(const orc_room* room, const positionAndRotation* cfg, resultCosts* out) {
    costs_ex(room, cfg, out, 1);
}

static void costs_ex(const orc_room* room, const positionAndRotation* cfg, resultCosts* out,
                     int with_ol) {
    const Surface* s = room->srf;
    float pw = (float)(orc_pairwise(room, cfg) * orc_pairwise_angle(room, cfg));
    out->PairWiseCosts = s->WeightPairWise * pw;
    float vb = (float)orc_visual_balance(room, cfg);
    out->VisualBalanceCosts = s->WeightVisualBalance * vb;
    float fp = (float)orc_focal_point(room, cfg);
    out->FocalPointCosts = s->WeightFocalPoint * fp;
    float sym = orc_symmetry(room, cfg);
    out->SymmetryCosts = s->WeightSymmetry * sym;
    float ol = with_ol ? orc_off_limits(room, cfg) : 0.0f;
    out->OffLimitsCosts = s->WeightOffLimits * ol;
    float cl = orc_clearance(room, cfg);
    out->ClearanceCosts = s->WeightClearance * cl;
    float sa = orc_surface_area(room, cfg);
    out->SurfaceAreaCosts = s->WeightSurfaceArea * sa;
    float t = out->PairWiseCosts + out->VisualBalanceCosts;
    t = t + out->FocalPointCosts;
    t = t + out->SymmetryCosts;
    t = t + out->ClearanceCosts;
    t = t + out->SurfaceAreaCosts;
    out->totalCosts = t;
}

/* ------------------------------------------------------------------------------------------
 * MH step, Kernel.cu:566-713.
 * ---------------------------------------------------------------------------------------- */

/* Kernel.cu:566-574: u in (0,1] scaled by (max - min + 0.999999) in double, kept as a float,
 * truncated. With max = nObjs - 1 >= 63, u == 1.0f yields nObjs. */
static int rand_int(orc_rng* r, int max, int min) {
    float u = orc_rng_uniform(r);
    u = (float)((double)u * ((double)(max - min) + 0.999999));
    u = u + (float)min;
    return (int)truncf(u);
}

int orc_rand_int(orc_rng* r, int max, int min) { return rand_int(r, max, min); }

/* Draws of index nObjs seen by pick_object in this process (test diagnostic: lets a test
 * prove that a fixture exercises the u == 1.0f edge of Kernel.cu:566-574). */
static long long g_index_n_draws;

long long orc_index_n_draws(int reset) {
    const long long v = __atomic_load_n(&g_index_n_draws, __ATOMIC_RELAXED);
    if (reset) __atomic_store_n(&g_index_n_draws, 0, __ATOMIC_RELAXED);
    return v;
}

/* Object pick with redraw while frozen (Kernel.cu:598-602); index nObjs is frozen. */
static int pick_object(const positionAndRotation* cfg, int n, orc_rng* r) {
    int k = rand_int(r, n - 1, 0);
    for (;;) {
        if (k >= n) __atomic_add_fetch(&g_index_n_draws, 1, __ATOMIC_RELAXED);
        else if (!cfg[k].frozen) break;
        k = rand_int(r, n - 1, 0);
    }
    return k;
}

int orc_pick_object(const positionAndRotation* cfg, int n, orc_rng* r) {
    return pick_object(cfg, n, r);
}

void orc_propose(const orc_room* room, positionAndRotation* cfg, orc_rng* r) {
    const int n = room->srf->nObjs;
    int mode = rand_int(r, 2, 0);
    dvec2 rmin = aabb_min(room->surfaceRectangle, 0, 0, 0);
    dvec2 rmax = aabb_max(room->surfaceRectangle, 0, 0, 0);
    float width = (float)(rmax.x - rmin.x);
    float height = (float)(rmax.y - rmin.y);
    float sx = width / 16;
    float sy = height / 16;
    if (mode == 0) { /* translate, Kernel.cu:595-632 */
        int k = pick_object(cfg, n, r);
        float dx = orc_rng_normal(r);
        dx = dx * sx;
        float dy = orc_rng_normal(r);
        dy = dy * sy;
        positionAndRotation* o = &cfg[k];
        if (o->x + dx > rmax.x) o->x = rmax.x;
        else if (o->x + dx < rmin.x) o->x = rmin.x;
        else o->x = o->x + dx;
        if (o->y + dy > rmax.y) o->y = rmax.y;
        else if (o->y + dy < rmin.y) o->y = rmin.y;
        else o->y = o->y + dy;
    } else if (mode == 1) { /* rotate, Kernel.cu:634-653 */
        int k = pick_object(cfg, n, r);
        float dr = orc_rng_normal(r);
        dr = (float)(dr * ORC_S_SIGMA_T);
        positionAndRotation* o = &cfg[k];
        o->rotY = o->rotY + dr;
        if (o->rotY < 0) o->rotY = o->rotY + 2 * ORC_PI;
        else if (o->rotY > 2 * ORC_PI) o->rotY = o->rotY - 2 * ORC_PI;
    } else { /* swap, Kernel.cu:655-703; object 1's pose travels through floats */
        if (n < 2) return;
        int a = pick_object(cfg, n, r);
        int b = pick_object(cfg, n, r);
        positionAndRotation* p = &cfg[a];
        positionAndRotation* q = &cfg[b];
        float t[6] = {(float)p->x, (float)p->y, (float)p->z,
                      (float)p->rotX, (float)p->rotY, (float)p->rotZ};
        p->x = q->x; p->y = q->y; p->z = q->z;
        p->rotX = q->rotX; p->rotY = q->rotY; p->rotZ = q->rotZ;
        q->x = t[0]; q->y = t[1]; q->z = t[2];
        q->rotX = t[3]; q->rotY = t[4]; q->rotZ = t[5];
    }
}

/* Accept draws of u == 1.0f (the (0,1] uniform's top value) against an uphill proposal, whose
 * threshold min(1, exp(...)) is exactly 1 and so rejects it (test diagnostic: lets a test prove
 * that a fixture exercises this edge of Kernel.cu:706-713). */
static long long g_u1_uphill;

long long orc_u1_uphill_draws(int reset) {
    const long long v = __atomic_load_n(&g_u1_uphill, __ATOMIC_RELAXED);
    if (reset) __atomic_store_n(&g_u1_uphill, 0, __ATOMIC_RELAXED);
    return v;
}

/* Kernel.cu:706-713: maximises the total; exp in double, rounded to float. */
int orc_accept(double cost_star, double cost_cur, orc_rng* r) {
    float u = orc_rng_uniform(r);
    float a = fminf(1.0f, (float)mh_exp(ORC_BETA * (cost_star - cost_cur)));
    return u < a;
}

/* Accept at inverse temperature beta (parallel tempering; beta = BETA is Accept itself). */
int orc_accept_at(double cost_star, double cost_cur, double beta, orc_rng* r) {
    float u = orc_rng_uniform(r);
    if (u == 1.0f && cost_star > cost_cur) __atomic_add_fetch(&g_u1_uphill, 1, __ATOMIC_RELAXED);
    float a = fminf(1.0f, (float)mh_exp(beta * (cost_star - cost_cur)));
    return u < a;
}

/* ------------------------------------------------------------------------------------------
 * Validation (the reference performs none; see mh_kernel.h).
 * ---------------------------------------------------------------------------------------- */
int orc_validate(const orc_room* room, const positionAndRotation* cfg) {
    const Surface* s = room->srf;
    if (!s) return fail("srf is NULL%ld", 0);
    const int n = s->nObjs, c = s->nClearances, nr = s->nRelationships;
    if (n < 1) return fail("nObjs must be >= 1 (got %ld)", n);
    if (c < 0 || c > n) return fail("nClearances must be in [0, nObjs] (got %ld)", c);
    if (nr < 0) return fail("nRelationships must be >= 0 (got %ld)", nr);
    if (!cfg || !room->offlimits || !room->vertices || !room->surfaceRectangle)
        return fail("NULL input array%ld", 0);
    if ((nr > 0 && (!room->rs || !room->ra)) || (c > 0 && !room->clearances))
        return fail("NULL input array%ld", 0);
    const long nv = 4L * (c + n);
    int any_free = 0;
    for (int i = 0; i < n; ++i) {
        int p = room->offlimits[i].point1Index;
        if (p < 0 || p + 3 >= nv) return fail("offlimits[%ld].point1Index out of range", i);
        if (!cfg[i].frozen) any_free = 1;
    }
    if (!any_free) return fail("every object is frozen (the reference never terminates)%ld", 0);
    for (int i = 0; i < c; ++i) {
        int p = room->clearances[i].point1Index, q = room->clearances[i].SourceIndex;
        if (p < 0 || p + 3 >= nv) return fail("clearances[%ld].point1Index out of range", i);
        if (q < 0 || q >= n) return fail("clearances[%ld].SourceIndex out of range", i);
    }
    for (int i = 0; i < nr; ++i) {
        if (room->rs[i].SourceIndex < 0 || room->rs[i].SourceIndex >= n ||
            room->rs[i].TargetIndex < 0 || room->rs[i].TargetIndex >= n)
            return fail("rss[%ld] index out of range", i);
        if (room->ra[i].SourceIndex < 0 || room->ra[i].SourceIndex >= n ||
            room->ra[i].TargetIndex < 0 || room->ra[i].TargetIndex >= n)
            return fail("rsa[%ld] index out of range", i);
    }
    g_err[0] = 0;
    return 0;
}

/* ------------------------------------------------------------------------------------------
 * Chains, Kernel.cu:777-828 with the defined semantics of the header.
 * ---------------------------------------------------------------------------------------- */
typedef struct {
    const orc_room* room;
    const positionAndRotation* cfg;
    uint64_t seed;
    int64_t chain_begin;
    int64_t lo, hi; /* local chain range for this worker */
    int iterations;
    int track; /* MH_TRACK_* */
    int rng;   /* MH_RNG_* */
    int n_temps, swap_interval;
    const double* ladder;
    point* out_points;
    positionAndRotation* out_state;
    resultCosts* out_costs;
    int64_t* out_accepted;
} chain_job;

/* One chain's state between steps. */
typedef struct {
    positionAndRotation *cur, *star, *best;
    resultCosts cc, bc;
    orc_rng r;
    int64_t acc;
    int rung;
} chain_state;

static void chain_alloc(chain_state* st, int n) {
    st->cur = malloc(sizeof(positionAndRotation) * n);
    st->star = malloc(sizeof(positionAndRotation) * n);
    st->best = malloc(sizeof(positionAndRotation) * n);
}

static void chain_free(chain_state* st) {
    free(st->cur);
    free(st->star);
    free(st->best);
}

static void chain_init(const chain_job* job, int64_t local, chain_state* st) {
    const int n = job->room->srf->nObjs;
    const uint64_t gid = (uint64_t)(job->chain_begin + local);
    if (job->rng == MH_RNG_CURAND_XORWOW) /* curand_init(seed + tid, tid, 0), Kernel.cu:159 */
        orc_rng_init_xorwow(&st->r, (uint32_t)(job->seed + gid), gid, ORC_XORWOW_CURAND);
    else
        orc_rng_init(&st->r, job->seed, gid);
    memcpy(st->cur, job->cfg, sizeof(positionAndRotation) * n);
    costs_ex(job->room, st->cur, &st->cc, g_step_offlimits);
    /* Best-of-chain, the reference's commented-out intent: cfgBest := cfgCurrent
     * (Kernel.cu:779-782); star replaces best when it improves, before Accept (:808-816). */
    st->bc = st->cc;
    if (job->track) memcpy(st->best, st->cur, sizeof(positionAndRotation) * n);
    st->acc = 0;
    st->rung = 0;
}

/* `steps` iterations of Kernel.cu:785-828 (full copies) at inverse temperature beta. */
static void chain_steps(const chain_job* job, chain_state* st, int steps, double beta) {
    const int n = job->room->srf->nObjs;
    resultCosts sc;
    for (int it = 0; it < steps; ++it) {
        memcpy(st->star, st->cur, sizeof(positionAndRotation) * n);
        orc_propose(job->room, st->star, &st->r);
        costs_ex(job->room, st->star, &sc, g_step_offlimits);
        if (job->track && (job->track == MH_TRACK_LOWEST ? sc.totalCosts < st->bc.totalCosts
                                                         : sc.totalCosts > st->bc.totalCosts)) {
            memcpy(st->best, st->star, sizeof(positionAndRotation) * n);
            st->bc = sc;
        }
        if (orc_accept_at(sc.totalCosts, st->cc.totalCosts, beta, &st->r)) {
            positionAndRotation* t = st->cur;
            st->cur = st->star;
            st->star = t;
            st->cc = sc;
            ++st->acc;
        }
    }
}

static void chain_output(const chain_job* job, const chain_state* st, int64_t slot,
                         int64_t local) {
    const int n = job->room->srf->nObjs;
    /* with tracking the output is cfgBest / bestCosts (Kernel.cu:840-860, commented out) */
    const positionAndRotation* out = job->track ? st->best : st->cur;
    resultCosts oc = job->track ? st->bc : st->cc;
    if (!g_step_offlimits)  /* the output configuration's own OffLimits (see g_step_offlimits) */
        oc.OffLimitsCosts = job->room->srf->WeightOffLimits * orc_off_limits(job->room, out);
    if (job->out_points) {
        point* p = job->out_points + slot * n;
        for (int i = 0; i < n; ++i) {
            p[i].x = (float)out[i].x; p[i].y = (float)out[i].y; p[i].z = (float)out[i].z;
            p[i].rotX = (float)out[i].rotX; p[i].rotY = (float)out[i].rotY;
            p[i].rotZ = (float)out[i].rotZ;
        }
    }
    if (job->out_state) memcpy(job->out_state + slot * n, out, sizeof(positionAndRotation) * n);
    if (job->out_costs) job->out_costs[slot] = oc;
    if (job->out_accepted) job->out_accepted[local] = st->acc;
}

static void run_one(const chain_job* job, int64_t local, chain_state* st) {
    chain_init(job, local, st);
    chain_steps(job, st, job->iterations, ORC_BETA);
    chain_output(job, st, local, local);
}

/* Parallel tempering (mh_options.n_temps = K > 1): group g = local chains [g*K, (g+1)*K).
 * Replicas step independently at their rung's beta; after every swap_interval steps, exchange
 * round t tries the rung pairs (k, k+1), k = (t-1) mod 2 + 2i, with the Philox uniform of
 * (seed, subsequence 2^63 + global group, offset (t-1)*K + k) against
 * min(1, (float)exp((beta_k - beta_k+1) * (E_k+1 - E_k))). Output slot g*K + final rung. */
static void run_group(const chain_job* job, int64_t g, chain_state* st) {
    const int K = job->n_temps;
    int perm[1024];
    for (int j = 0; j < K; ++j) {
        chain_init(job, g * K + j, &st[j]);
        st[j].rung = j;
        perm[j] = j;
    }
    const uint64_t gid = (uint64_t)(job->chain_begin / K + g);
    int64_t done = 0;
    while (done < job->iterations) {
        int chunk = job->iterations - (int)done;
        const int to_round = job->swap_interval - (int)(done % job->swap_interval);
        if (to_round < chunk) chunk = to_round;
        for (int j = 0; j < K; ++j) chain_steps(job, &st[j], chunk, job->ladder[st[j].rung]);
        done += chunk;
        if (done % job->swap_interval == 0) {
            const int64_t round = done / job->swap_interval;
            for (int k = (int)((round - 1) & 1); k + 1 < K; k += 2) {
                const int ca = perm[k], cb = perm[k + 1];
                orc_rng u_r;
                orc_rng_init_offset(&u_r, job->seed, (1ull << 63) | gid,
                                    (uint64_t)(round - 1) * K + k);
                const float u = orc_rng_uniform(&u_r);
                const double db = job->ladder[k] - job->ladder[k + 1];
                const float thr = fminf(1.0f, (float)mh_exp(db * ((double)st[cb].cc.totalCosts -
                                                               (double)st[ca].cc.totalCosts)));
                if (u < thr) {
                    perm[k] = cb;
                    perm[k + 1] = ca;
                    st[ca].rung = k + 1;
                    st[cb].rung = k;
                }
            }
        }
    }
    for (int j = 0; j < K; ++j) chain_output(job, &st[j], g * K + st[j].rung, g * K + j);
}

static void* chain_worker(void* arg) {
    const chain_job* job = (const chain_job*)arg;
    const int n = job->room->srf->nObjs;
    const int K = job->n_temps > 1 ? job->n_temps : 1;
    chain_state* st = calloc((size_t)K, sizeof(chain_state));
    for (int j = 0; j < K; ++j) chain_alloc(&st[j], n);
    if (K > 1)  /* lo/hi count groups */
        for (int64_t g = job->lo; g < job->hi; ++g) run_group(job, g, st);
    else
        for (int64_t c = job->lo; c < job->hi; ++c) run_one(job, c, &st[0]);
    for (int j = 0; j < K; ++j) chain_free(&st[j]);
    free(st);
    return NULL;
}

static int run_chains(const orc_room* room, const positionAndRotation* cfg, const mh_options* o,
                      int64_t chain_begin, int64_t n_chains, int iterations, int nthreads,
                      point* out_points, positionAndRotation* out_state,
                      resultCosts* out_costs, int64_t* out_accepted) {
    if (orc_validate(room, cfg) != 0) return -1;
    if (n_chains < 0 || iterations < 0) return fail("negative chain or step count%ld", 0);
    if (o->track_best < MH_TRACK_OFF || o->track_best > MH_TRACK_HIGHEST)
        return fail("bad track_best %ld", o->track_best);
    if (o->rng < MH_RNG_PHILOX || o->rng > MH_RNG_CURAND_XORWOW) return fail("bad rng %ld", o->rng);
    const int K = o->n_temps > 1 ? o->n_temps : 1;
    if (K > 1024) return fail("n_temps %ld > 1024", K);
    if (K > 1 && (n_chains % K || chain_begin % K || o->swap_interval < 1 ||
                  !(o->beta_min > 0.0) || !(o->beta_min <= ORC_BETA)))
        return fail("bad parallel tempering options (n_temps %ld)", K);
    double ladder[1024];
    for (int k = 0; k < K; ++k) /* geometric from BETA (rung 0) down to beta_min */
        ladder[k] = k == 0 ? ORC_BETA : ORC_BETA * pow(o->beta_min / ORC_BETA, (double)k / (K - 1));
    const int64_t units = n_chains / K; /* chains, or tempering groups */
    if (nthreads < 1) nthreads = 1;
    if (nthreads > units) nthreads = (int)(units > 0 ? units : 1);
    chain_job* jobs = calloc((size_t)nthreads, sizeof(chain_job));
    pthread_t* th = calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; ++t) {
        chain_job j = {room, cfg, o->seed, chain_begin,
                       units * t / nthreads, units * (t + 1) / nthreads,
                       iterations, o->track_best, o->rng, K, o->swap_interval, ladder,
                       out_points, out_state, out_costs, out_accepted};
        jobs[t] = j;
    }
    for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, chain_worker, &jobs[t]);
    chain_worker(&jobs[0]);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
    free(jobs);
    free(th);
    return 0;
}

static mh_options plain_options(uint64_t seed) {
    mh_options o;
    memset(&o, 0, sizeof o);
    o.seed = seed;
    o.n_temps = 1;
    o.swap_interval = 1;
    o.beta_min = ORC_BETA;
    return o;
}

int orc_run_chains(const orc_room* room, const positionAndRotation* cfg, uint64_t seed,
                   int64_t chain_begin, int64_t n_chains, int iterations, int nthreads,
                   point* out_points, resultCosts* out_costs, int64_t* out_accepted) {
    const mh_options o = plain_options(seed);
    return run_chains(room, cfg, &o, chain_begin, n_chains, iterations, nthreads, out_points,
                      NULL, out_costs, out_accepted);
}

int orc_run_chains_state(const orc_room* room, const positionAndRotation* cfg, uint64_t seed,
                         int64_t chain_begin, int64_t n_chains, int iterations, int nthreads,
                         positionAndRotation* out_state, resultCosts* out_costs,
                         int64_t* out_accepted) {
    const mh_options o = plain_options(seed);
    return run_chains(room, cfg, &o, chain_begin, n_chains, iterations, nthreads, NULL,
                      out_state, out_costs, out_accepted);
}

int orc_run_chains_ex(const orc_room* room, const positionAndRotation* cfg,
                      const mh_options* opts, int64_t chain_begin, int64_t n_chains,
                      int iterations, int nthreads, positionAndRotation* out_state,
                      resultCosts* out_costs, int64_t* out_accepted) {
    return run_chains(room, cfg, opts, chain_begin, n_chains, iterations, nthreads, NULL,
                      out_state, out_costs, out_accepted);
}

/* ------------------------------------------------------------------------------------------
 * Numerics probes (tests/test_gpu_math.py): the shared math functions on the argument streams
 * of mh_math.h, and the C library's functions on the same arguments for comparison.
 * ---------------------------------------------------------------------------------------- */
static void probe_libm(int fn, uint64_t i, double* out) {
    const uint32_t w = (uint32_t)i;
    float y, x;
    switch (fn) {
        case MH_PROBE_BM_LOG: out[0] = log((double)w * 0x1p-32 + 0x1p-33); break;
        case MH_PROBE_BM_SINCOS: {
            const double a = 6.283185307179586 * ((double)w * 0x1p-32 + 0x1p-33);
            out[0] = sin(a);
            out[1] = cos(a);
            break;
        }
        case MH_PROBE_COS_F32: {
            float v;
            memcpy(&v, &w, 4);
            out[0] = (double)(float)cos((double)v);
            break;
        }
        case MH_PROBE_XW_LOG:
            out[0] = (double)(float)log((double)((float)w * 0x1p-32f + 0x1p-32f * 0.5f));
            break;
        case MH_PROBE_XW_SINCOS: {
            const float k = 0x1p-32f * 6.2831855f;
            const double v = (double)fmaf((float)w, k, k * 0.5f);
            out[0] = sin(v);
            out[1] = cos(v);
            break;
        }
        case MH_PROBE_ATAN2_ROOM:
        case MH_PROBE_ATAN2_BITS:
            mh_arg_atan2(i, fn == MH_PROBE_ATAN2_BITS, &y, &x);
            out[0] = atan2((double)y, (double)x);
            break;
        case MH_PROBE_ATAN2F_ROOM:
        case MH_PROBE_ATAN2F_BITS:
            mh_arg_atan2(i, fn == MH_PROBE_ATAN2F_BITS, &y, &x);
            out[0] = (double)(float)atan2((double)y, (double)x);
            break;
        case MH_PROBE_ACCEPT: {
            float u;
            double xa;
            mh_arg_accept(i, &u, &xa);
            const float e = xa >= 0.0 ? 1.0f : xa < -24.0 ? 0.0f : fminf(1.0f, (float)exp(xa));
            out[0] = u < e ? 1.0 : 0.0;
            break;
        }
        default: out[0] = exp(mh_arg_exp(i, fn == MH_PROBE_EXP_ANY)); break;
    }
}

typedef struct {
    int fn, libm;
    uint64_t start, count;
    double* out;
} probe_job;

static void* probe_worker(void* arg) {
    const probe_job* j = (const probe_job*)arg;
    const int w = mh_probe_width(j->fn);
    for (uint64_t k = 0; k < j->count; ++k) {
        if (j->libm) probe_libm(j->fn, j->start + k, j->out + k * w);
        else mh_math_probe(j->fn, j->start + k, j->out + k * w);
    }
    return NULL;
}

static int probe_run(int fn, int libm, uint64_t start, uint64_t count, int nthreads, double* out) {
    if (fn < 0 || fn >= MH_PROBE_COUNT || !out) return fail("bad probe %ld", fn);
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    probe_job jobs[256];
    const int w = mh_probe_width(fn);
    for (int t = 0; t < nthreads; ++t) {
        const uint64_t b = count * (uint64_t)t / (uint64_t)nthreads;
        const uint64_t e = count * (uint64_t)(t + 1) / (uint64_t)nthreads;
        jobs[t].fn = fn;
        jobs[t].libm = libm;
        jobs[t].start = start + b;
        jobs[t].count = e - b;
        jobs[t].out = out + b * w;
    }
    for (int t = 1; t < nthreads; ++t) pthread_create(&th[t], NULL, probe_worker, &jobs[t]);
    probe_worker(&jobs[0]);
    for (int t = 1; t < nthreads; ++t) pthread_join(th[t], NULL);
    return 0;
}

int orc_math_eval(int fn, uint64_t start, uint64_t count, int nthreads, double* out) {
    return probe_run(fn, 0, start, count, nthreads, out);
}

int orc_math_eval_libm(int fn, uint64_t start, uint64_t count, int nthreads, double* out) {
    return probe_run(fn, 1, start, count, nthreads, out);
}

/* mh_math.h's functions on given arguments (tests/test_math.py measures their accuracy):
 * which = 0 log, 1 exp, 2 sin, 3 cos, 4 atan2(a, b), 5 sin of the medium reduction only. */
int orc_math_apply(int which, const double* a, const double* b, int64_t n, double* out) {
    if (which < 0 || which > 5 || !a || !out || (which == 4 && !b)) return fail("bad function %ld", which);
    for (int64_t i = 0; i < n; ++i) {
        double sn, cs;
        switch (which) {
            case 0: out[i] = mh_log(a[i]); break;
            case 1: out[i] = mh_exp(a[i]); break;
            case 2: out[i] = mh_sin(a[i]); break;
            case 3: out[i] = mh_cos(a[i]); break;
            case 4: out[i] = mh_atan2(a[i], b[i]); break;
            default: mh_sincos_medium(a[i], &sn, &cs); out[i] = sn; break;
        }
    }
    return 0;
}
