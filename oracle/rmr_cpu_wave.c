/*
 * oracle/rmr_cpu_wave.c — CPU BASELINE (bench.py's cpu_baseline leg; test infrastructure, never the
 * product path): the oracle's RM1 path (RayMarch.glsl main -> trace -> march -> map, RM1:483-612)
 * run 8 paths at a time on AVX2, the way the reference's own CPU path runs on Mesa llvmpipe (its
 * JIT executes 8 shader invocations per 256-bit vector).
 *
 * Each of the VW SIMD lanes holds one independent path (one pixel sample), a state machine like the
 * GPU kernel's lane: every loop iteration evaluates map() (RM1:224-231) for all VW lanes at once —
 * a march step (RM1:233-257) or a getNormal probe (RM1:259-268) — and updates the march state as
 * vectors; a lane whose march or normal finishes runs its shading (materials, RNG, bounce logic)
 * with the oracle's own scalar functions, and a lane whose sample is done takes the next one.
 *
 * Results are bitwise those of oracle/rmr_oracle.c (tests/test_cpu_wave.py): the same IEEE operations
 * per lane (contraction off; fmaf -> vfmadd; sqrtf -> vsqrtps, both correctly rounded; glibc's
 * fmaxf / fminf, which return the second operand on equality, -> vmaxps / vminps, with the NaN
 * operand rule of fmaxf restored where an operand can be NaN), the same RNG call order (shading is
 * the scalar oracle code), and the running mean folded in sample order.
 * RM2 / RM3 scenes are not handled here (oracle_render_wave returns -1; the caller times the scalar
 * oracle).
 */
#include "rmr_oracle.c"

#include <immintrin.h>

#define VW 8

typedef __m256 vf;

/* fmaxf(a, b) of glibc: a > b ? a : b, the other operand where one is NaN */
static inline vf vfmaxf(vf a, vf b) {
    const vf m = _mm256_max_ps(a, b);                        /* a > b ? a : b (NaN a: b) */
    return _mm256_blendv_ps(m, a, _mm256_cmp_ps(b, b, _CMP_UNORD_Q));   /* NaN b: a */
}
static inline vf vabs(vf a) { return _mm256_andnot_ps(_mm256_set1_ps(-0.0f), a); }
/* v_dot(v, v) = fmaf(x, x, fmaf(y, y, z * z)) */
static inline vf vdot3(vf x, vf y, vf z) {
    return _mm256_fmadd_ps(x, x, _mm256_fmadd_ps(y, y, _mm256_mul_ps(z, z)));
}

/* o_map (RM1:224-231 + the opU NaN rule) for VW points; inactive lanes compute garbage */
static void map_vec(const rmr_scene* sc, float max_dist, const float* px, const float* py, const float* pz,
                    float* dist, float* id) {
    const vf X = _mm256_loadu_ps(px), Y = _mm256_loadu_ps(py), Z = _mm256_loadu_ps(pz);
    vf dx = _mm256_set1_ps(max_dist), dy = _mm256_set1_ps(-1.0f);
    for (int j = 0; j < sc->n_prims; j++) {
        const rmr_prim* pr = &sc->prims[j];
        vf dj;
        if (pr->type == RMR_PRIM_SPHERE) {   /* sd_sphere: length(p - c) - r */
            const vf vx = _mm256_sub_ps(X, _mm256_set1_ps(pr->c[0]));
            const vf vy = _mm256_sub_ps(Y, _mm256_set1_ps(pr->c[1]));
            const vf vz = _mm256_sub_ps(Z, _mm256_set1_ps(pr->c[2]));
            dj = _mm256_sub_ps(_mm256_sqrt_ps(vdot3(vx, vy, vz)), _mm256_set1_ps(pr->r[0]));
        } else if (pr->type == RMR_PRIM_BOX) {   /* sd_box: min(max(q), 0) + length(max(q, 0)) */
            const vf qx = _mm256_sub_ps(vabs(_mm256_sub_ps(X, _mm256_set1_ps(pr->c[0]))), _mm256_set1_ps(pr->r[0]));
            const vf qy = _mm256_sub_ps(vabs(_mm256_sub_ps(Y, _mm256_set1_ps(pr->c[1]))), _mm256_set1_ps(pr->r[1]));
            const vf qz = _mm256_sub_ps(vabs(_mm256_sub_ps(Z, _mm256_set1_ps(pr->c[2]))), _mm256_set1_ps(pr->r[2]));
            const vf zero = _mm256_setzero_ps();
            /* fminf(M, 0) and fmaxf(q, 0): the constant second operand is never NaN */
            const vf k = _mm256_min_ps(vfmaxf(qx, vfmaxf(qy, qz)), zero);
            const vf ox = _mm256_max_ps(qx, zero), oy = _mm256_max_ps(qy, zero), oz = _mm256_max_ps(qz, zero);
            dj = _mm256_add_ps(k, _mm256_sqrt_ps(vdot3(ox, oy, oz)));
        } else {   /* Mandelbulb / node programs: the oracle's scalar prim_dist per lane */
            float x[VW], y[VW], z[VW], r[VW];
            _mm256_storeu_ps(x, X);
            _mm256_storeu_ps(y, Y);
            _mm256_storeu_ps(z, Z);
            for (int l = 0; l < VW; l++) r[l] = prim_dist(sc, pr, o3(x[l], y[l], z[l]));
            dj = _mm256_loadu_ps(r);
        }
        /* opU: id when !(d.x < dj), distance when d.x >= dj (o_map) */
        const vf take_id = _mm256_cmp_ps(dx, dj, _CMP_NLT_UQ);
        const vf take_d = _mm256_cmp_ps(dx, dj, _CMP_GE_OQ);
        dy = _mm256_blendv_ps(dy, _mm256_set1_ps(pr->mat_id), take_id);
        dx = _mm256_blendv_ps(dx, dj, take_d);
    }
    _mm256_storeu_ps(dist, dx);
    _mm256_storeu_ps(id, dy);
}

enum { W_IDLE = 0, W_MARCH = 1, W_NORMAL = 2 };

/* the part of a lane that only shading reads (AoS); the march state is SoA in `wave` */
typedef struct wpath {
    lane L;            /* the oracle's invocation state: RNG chain, channels, map counter */
    long unit;         /* sample index in the chunk's unit list */
    int px, py;
    o_v3 dir0;         /* primary direction (separateChannels restarts, RM1:586-598) */
    int chan;          /* -1, or the channel pass 0..2 */
    o_v3 acc;          /* separateChannels: r, then r + g */
    o_v3 color, o, d;  /* trace_rm1 locals */
    int inside, bounces;
    o_v2 v;            /* march result */
    o_v3 hit;
} wpath;

typedef struct wave {
    wpath p[VW];
    int phase[VW];
    /* march point = fma(d, t, o); probe point = hit + e */
    float ox[VW], oy[VW], oz[VW], dx[VW], dy[VW], dz[VW], t[VW], dm[VW];
    int step[VW];
    float hx[VW], hy[VW], hz[VW], ex[VW], ey[VW], ez[VW];
    int probe[VW];
    float pm[6][VW];
} wave;

/* one batch of pixels [i0, i0 + npx) of the rect (row-major, width w) x nspp samples, shared by the
 * threads: each thread's wave takes the next unit from `next` (atomic) whenever a lane is free, so the
 * lanes drain once per batch, not once per thread's share */
typedef struct wctx {
    const oracle_job* job;
    const float* times;
    int x0, w;
    long i0;
    int y0;
    const int* rows;    /* the rect's rows (NULL: y0, y0 + 1, ...) */
    uint32_t nspp;
    long next, total;   /* units handed out (shared) / in the batch */
    float* res;         /* [npx * nspp][3] sample radiance */
} wctx;

static void set_march(wave* w, int l) {
    wpath* P = &w->p[l];
    w->ox[l] = P->o.x; w->oy[l] = P->o.y; w->oz[l] = P->o.z;
    w->dx[l] = P->d.x; w->dy[l] = P->d.y; w->dz[l] = P->d.z;
    w->t[l] = 0.0f;
    w->step[l] = 0;
    w->dm[l] = P->inside ? -1.0f : 1.0f;
    w->phase[l] = W_MARCH;
}

static void after_march(wctx* c, wave* w, int l);
static void finish_trace(wctx* c, wave* w, int l, o_v3 col);
static void start_trace(wctx* c, wave* w, int l, o_v3 eye, o_v3 dir);

/* trace_rm1's `while (bounces < maxBounces) { bounces++; march ... }` */
static void next_bounce(wctx* c, wave* w, int l) {
    wpath* P = &w->p[l];
    if (P->bounces < P->L.max_bounces) {
        P->bounces++;
        if (P->L.max_steps <= 0) {   /* o_march's loop does not run: the miss */
            P->v = o2(P->L.max_dist, -1.0f);
            after_march(c, w, l);
        } else {
            set_march(w, l);
        }
    } else {
        finish_trace(c, w, l, P->color);
    }
}

static void start_trace(wctx* c, wave* w, int l, o_v3 eye, o_v3 dir) {
    wpath* P = &w->p[l];
    P->color = P->L.channels;
    P->o = eye;
    P->d = dir;
    P->inside = 0;
    P->bounces = 0;
    next_bounce(c, w, l);
}

/* a fresh sample for the idle lane l (sample_rgb's jittered primary ray, RM1:569-584); false when the
 * batch has none left. The sample may finish at once (maxBounces 0, maxSteps 0: the lane is idle
 * again), so callers refill in a loop (refill) rather than by recursion */
static int take_unit(wctx* c, wave* w, int l) {
    const long u = __atomic_fetch_add(&c->next, 1, __ATOMIC_RELAXED);
    if (u >= c->total) return 0;
    const long pi = u / c->nspp;
    const uint32_t k = (uint32_t)(u % c->nspp);
    const long gi = c->i0 + pi;
    const int px = c->x0 + (int)(gi % c->w), py = c->rows ? c->rows[gi / c->w] : c->y0 + (int)(gi / c->w);
    wpath* P = &w->p[l];
    lane_init(&P->L, c->job, px, py, c->times[k]);
    P->unit = u;
    P->px = px;
    P->py = py;
    const oracle_job* job = c->job;
    const float* V = job->view;
    const o_v3 eye = o3(V[0], V[1], V[2]);
    const o_v3 r00 = o3(V[3], V[4], V[5]), r01 = o3(V[6], V[7], V[8]);
    const o_v3 r10 = o3(V[9], V[10], V[11]), r11 = o3(V[12], V[13], V[14]);
    const float W = (float)job->W, H = (float)job->H;
    const float posx = (float)px / W, posy = (float)py / H;
    const float t = P->L.time;
    const float j1 = o_rand(&P->L, o2((float)px + t, (float)py + t));
    const float j2 = o_rand(&P->L, o2((float)px + t, (float)py + t));
    const float j3 = o_rand(&P->L, o2((float)py + t, (float)px + t));
    const o_v3 top = v_mix(r00, r01, posx + j1 / W);
    const o_v3 bot = v_mix(r10, r11, posx + j2 / W);
    P->dir0 = v_normalize(v_mix(top, bot, posy + j3 / H));
    if (job->params.separate_channels == 0) {
        P->chan = -1;
        P->L.channels = o3s(1.0f);
    } else {
        P->chan = 0;
        P->L.channels = o3(1.0f, 0.0f, 0.0f);
    }
    start_trace(c, w, l, eye, P->dir0);
    return 1;
}
static void refill(wctx* c, wave* w, int l) {
    while (w->phase[l] == W_IDLE && take_unit(c, w, l)) {
    }
}

/* end of trace(): the sample (or the next separateChannels pass, sample_rgb); the lane is then idle */
static void finish_trace(wctx* c, wave* w, int l, o_v3 col) {
    wpath* P = &w->p[l];
    if (P->chan >= 0) {
        P->acc = P->chan == 0 ? col : v_add(P->acc, col);
        if (P->chan < 2) {
            P->chan++;
            P->L.channels = o3(P->chan == 0 ? 1.0f : 0.0f, P->chan == 1 ? 1.0f : 0.0f, P->chan == 2 ? 1.0f : 0.0f);
            const float* V = c->job->view;
            start_trace(c, w, l, o3(V[0], V[1], V[2]), P->dir0);
            return;
        }
        col = P->acc;
    }
    float* r = c->res + 3 * P->unit;
    r[0] = col.x; r[1] = col.y; r[2] = col.z;
    w->phase[l] = W_IDLE;
}

/* trace_rm1 after march(): hit -> getNormal probes, miss -> sky (RM1:514-561) */
static void after_march(wctx* c, wave* w, int l) {
    wpath* P = &w->p[l];
    P->hit = v_fma(P->d, P->v.x, P->o);
    if (P->v.x < P->L.max_dist) {
        w->hx[l] = P->hit.x; w->hy[l] = P->hit.y; w->hz[l] = P->hit.z;
        w->ex[l] = 0.001f; w->ey[l] = 0.0f; w->ez[l] = 0.0f;   /* probe 0: (p.x + h, p.y + 0, p.z + 0) */
        w->probe[l] = 0;
        w->phase[l] = W_NORMAL;
        return;
    }
    const o_v3 emit = v_scale(sky_color(&P->L, P->d), gray1(&P->L, v_mul(o3s(1.0f), P->L.channels)));
    finish_trace(c, w, l, v_mul(P->color, emit));
}

/* the hit's material and the next bounce (RM1:515-553), N = getNormal(hit) */
static void shade_hit(wctx* c, wave* w, int l) {
    wpath* P = &w->p[l];
    const rmr_scene* sc = P->L.sc;
    const o_v3 N = v_normalize(o3(w->pm[0][l] - w->pm[1][l], w->pm[2][l] - w->pm[3][l], w->pm[4][l] - w->pm[5][l]));
    ray_data ray;
    ray.origin = P->o; ray.dir = P->d; ray.t = P->v.x; ray.hit = P->hit; ray.inside = P->inside;
    o_v3 nc = o3s(0), nd = o3s(0), ni = o3s(0), nh = o3s(0);
    const int id = (int)P->v.y;
    if (id >= 0 && id < sc->n_materials && sc->materials[id].defined)
        mat_v1(&P->L, &sc->materials[id], &ray, N, &nc, &nd, &ni, &nh);
    P->color = v_mul(P->color, nc);
    P->inside = ni.x != 0.0f;
    if (v_is_zero(nd)) {
        finish_trace(c, w, l, P->color);
        return;
    }
    P->d = nd;
    if (v_is_zero(nh)) P->o = P->inside ? v_fma(N, -0.002f, ray.hit) : v_fma(N, 0.003f, ray.hit);
    else P->o = nh;
    next_bounce(c, w, l);
}

/* getNormal's probe offsets in o_normal's order: +x, -x, +y, -y, +z, -z, as p + e (x - h == x + (-h);
 * y - 0 == y + (-0) and y + 0 == y + (+0) bit for bit, signed zeros included) */
static const float kProbe[6][3] = {{0.001f, 0.0f, 0.0f},  {-0.001f, -0.0f, -0.0f}, {0.0f, 0.001f, 0.0f},
                                   {-0.0f, -0.001f, -0.0f}, {0.0f, 0.0f, 0.001f},  {-0.0f, -0.0f, -0.001f}};

static uint64_t run_chunk(wctx* c) {
    wave w;
    memset(&w, 0, sizeof w);
    for (int l = 0; l < VW; l++) refill(c, &w, l);
    const oracle_job* job = c->job;
    const float max_dist = job->params.max_dist, step_mult = job->params.step_multiply;
    const int max_steps = job->params.max_steps;
    const vf vmax = _mm256_set1_ps(max_dist), vstep = _mm256_set1_ps(step_mult), vhit = _mm256_set1_ps(0.001f);
    uint64_t maps = 0;
    for (;;) {
        int any = 0, nmap = 0;
        for (int l = 0; l < VW; l++) {
            any |= w.phase[l];
            nmap += w.phase[l] != W_IDLE;
        }
        if (!any) break;
        maps += (uint64_t)nmap;
        /* the map() points: march fma(d, t, o) (v_fma), probe hit + e */
        float px[VW], py[VW], pz[VW], md[VW], mi[VW];
        {
            const vf T = _mm256_loadu_ps(w.t);
            const vf mx = _mm256_fmadd_ps(_mm256_loadu_ps(w.dx), T, _mm256_loadu_ps(w.ox));
            const vf my = _mm256_fmadd_ps(_mm256_loadu_ps(w.dy), T, _mm256_loadu_ps(w.oy));
            const vf mz = _mm256_fmadd_ps(_mm256_loadu_ps(w.dz), T, _mm256_loadu_ps(w.oz));
            const vf nx = _mm256_add_ps(_mm256_loadu_ps(w.hx), _mm256_loadu_ps(w.ex));
            const vf ny = _mm256_add_ps(_mm256_loadu_ps(w.hy), _mm256_loadu_ps(w.ey));
            const vf nz = _mm256_add_ps(_mm256_loadu_ps(w.hz), _mm256_loadu_ps(w.ez));
            const __m256i ph = _mm256_loadu_si256((const __m256i*)w.phase);
            const vf isn = _mm256_castsi256_ps(_mm256_cmpeq_epi32(ph, _mm256_set1_epi32(W_NORMAL)));
            _mm256_storeu_ps(px, _mm256_blendv_ps(mx, nx, isn));
            _mm256_storeu_ps(py, _mm256_blendv_ps(my, ny, isn));
            _mm256_storeu_ps(pz, _mm256_blendv_ps(mz, nz, isn));
        }
        map_vec(job->scene, max_dist, px, py, pz, md, mi);
        /* march(): m.x *= distMult; hit if < 0.001 (t returned); miss if t >= maxDist; else step */
        int ev = 0;
        {
            const vf T = _mm256_loadu_ps(w.t);
            const vf m = _mm256_mul_ps(_mm256_loadu_ps(md), _mm256_loadu_ps(w.dm));
            const vf hitm = _mm256_cmp_ps(m, vhit, _CMP_LT_OQ);
            const vf past = _mm256_cmp_ps(T, vmax, _CMP_GE_OQ);
            const vf tn = _mm256_fmadd_ps(m, vstep, T);
            const __m256i ph = _mm256_loadu_si256((const __m256i*)w.phase);
            const vf ism = _mm256_castsi256_ps(_mm256_cmpeq_epi32(ph, _mm256_set1_epi32(W_MARCH)));
            const vf stepping = _mm256_andnot_ps(_mm256_or_ps(hitm, past), ism);
            _mm256_storeu_ps(w.t, _mm256_blendv_ps(T, tn, stepping));
            const __m256i sn = _mm256_add_epi32(_mm256_loadu_si256((const __m256i*)w.step), _mm256_set1_epi32(1));
            _mm256_storeu_si256((__m256i*)w.step, _mm256_blendv_epi8(_mm256_loadu_si256((const __m256i*)w.step), sn,
                                                                      _mm256_castps_si256(stepping)));
            const vf lim = _mm256_castsi256_ps(_mm256_cmpgt_epi32(_mm256_set1_epi32(max_steps), sn));   /* step + 1 < maxSteps */
            /* a march lane ends on a hit, on t >= maxDist, or when its step count reaches maxSteps */
            const vf ends = _mm256_and_ps(ism, _mm256_or_ps(_mm256_or_ps(hitm, past), _mm256_andnot_ps(lim, stepping)));
            ev = _mm256_movemask_ps(ends);
            float hm[VW];
            _mm256_storeu_ps(hm, _mm256_and_ps(hitm, ism));
            for (int l = 0; l < VW; l++) {
                if (w.phase[l] == W_NORMAL) {
                    const int k = w.probe[l];
                    w.pm[k][l] = md[l];
                    if (k == 5) {
                        ev |= 1 << l;
                    } else {
                        w.probe[l] = k + 1;
                        w.ex[l] = kProbe[k + 1][0]; w.ey[l] = kProbe[k + 1][1]; w.ez[l] = kProbe[k + 1][2];
                    }
                } else if ((ev >> l) & 1) {
                    wpath* P = &w.p[l];
                    /* hit: (t, id) with t the march parameter before the step; else the miss */
                    P->v = hm[l] != 0.0f ? o2(T[l], mi[l]) : o2(max_dist, -1.0f);
                }
            }
        }
        while (ev) {
            const int l = __builtin_ctz((unsigned)ev);
            ev &= ev - 1;
            if (w.phase[l] == W_NORMAL) shade_hit(c, &w, l);
            else after_march(c, &w, l);
            refill(c, &w, l);
        }
    }
    return maps;
}

/* samples per batch (the result buffer: 12 B each) */
#define WAVE_BATCH (1L << 20)

/* oracle_render over the columns [x0, x1) of `nrows` rows (rows: the row indices, NULL = y0 ..
 * y0 + nrows - 1), RM1 scenes (same results bit for bit); -1 for RM2 / RM3 */
int oracle_render_wave_rows(const oracle_job* job, const float* times, int x0, int x1, int y0, const int* rows,
                            int nrows, uint32_t first_sample, uint32_t nspp, float* accum, int nthreads,
                            uint64_t* map_evals) {
    if (job->scene->variant != RMR_VARIANT_RM1) return -1;
    x0 = clampi(x0, 0, job->W); x1 = clampi(x1, 0, job->W);
    const int w = x1 - x0, h = nrows;
    if (w <= 0 || h <= 0 || nspp == 0) return 0;
    for (int r = 0; rows && r < nrows; r++)
        if (rows[r] < 0 || rows[r] >= job->H) return -2;
    const long npix = (long)w * h;
    long bpix = WAVE_BATCH / (long)nspp;
    if (bpix < 1) bpix = 1;
    float* res = (float*)malloc(sizeof(float) * 3 * (size_t)(bpix < npix ? bpix : npix) * nspp);
    uint64_t total = 0;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#endif
    for (long i0 = 0; i0 < npix; i0 += bpix) {
        const long n = npix - i0 < bpix ? npix - i0 : bpix;
        wctx c;
        c.job = job;
        c.times = times;
        c.x0 = x0;
        c.y0 = y0;
        c.rows = rows;
        c.w = w;
        c.i0 = i0;
        c.nspp = nspp;
        c.next = 0;
        c.total = n * (long)nspp;
        c.res = res;
#ifdef _OPENMP
#pragma omp parallel reduction(+ : total)
#endif
        total += run_chunk(&c);
#ifdef _OPENMP
#pragma omp parallel for schedule(static)
#endif
        for (long i = 0; i < n; i++) {   /* running mean in sample order (RM1:600-612) */
            const long gi = i0 + i;
            const int px = x0 + (int)(gi % w), py = rows ? rows[gi / w] : y0 + (int)(gi / w);
            float* acc = accum + 4 * ((long)py * job->W + px);
            for (uint32_t k = 0; k < nspp; k++) fold(acc, res + 3 * ((long)i * nspp + k), first_sample + k);
        }
    }
    free(res);
    if (map_evals) *map_evals += total;
    return 0;
}

/* oracle_render for RM1 scenes (same arguments and results, bit for bit); -1 for RM2 / RM3 */
int oracle_render_wave(const oracle_job* job, const float* times, int x0, int y0, int x1, int y1,
                       uint32_t first_sample, uint32_t nspp, float* accum, int nthreads, uint64_t* map_evals) {
    y0 = clampi(y0, 0, job->H);
    y1 = clampi(y1, 0, job->H);
    return oracle_render_wave_rows(job, times, x0, x1, y0, NULL, y1 - y0, first_sample, nspp, accum, nthreads, map_evals);
}
