/*
 * traversal_study.c — STUDY TOOL (test infrastructure, never linked into the product).
 *
 * Builds the oracle with a hook after every mesh walk (oracle.c mesh_bvh, path_tracer_kernel.cu:85-161)
 * and replays each walked ray through alternative traversals of the SAME BVH, counting the work
 * they do and every ray whose closest hit differs from the reference's preorder walk:
 *   oct     — stackless skip-index walk over a per-ray-octant copy of the tree whose children are
 *             ordered near-first along their split axis; cull `entry <= best`; ties on t broken by
 *             the reference preorder position of the leaf (the reference keeps the first in preorder).
 *   octm    — the same with the cull relaxed to entry <= best * (1 + 2^-10) (the detection margin).
 *   stack   — ordered BVH2 with a stack (test both children, descend the nearer): the ideal order.
 * An "anomaly" is a candidate triangle (test passes, t > 0) whose computed t lies before its leaf
 * box's computed entry: the only case in which the accepted hit can depend on visit order.
 *
 *   make -C tools study   then   python tools/traversal_study.py
 */
#include <stdint.h>
#include <stdio.h>
#include <string.h>

struct or_scene_fwd;
static void study_hook(const void* sc, int m, float ox, float oy, float oz, float dx, float dy, float dz, int hit,
                       float t, int tri);
#define OR_STUDY_HOOK(sc, m, o, d, hit, t, tri) study_hook(sc, m, o.x, o.y, o.z, d.x, d.y, d.z, hit, t, tri)
#include "../oracle/oracle.c"

typedef struct { float lo[3], hi[3]; int skip, tri, orig; } sn;
typedef struct { int n; int* left; int* right; sn* oct[8]; const pt_bvh_node_device* ref; unsigned long long* visits;
                 unsigned long long* passes; sn* meas; } smesh;

#define MAXM 16
static smesh g_mesh[MAXM];
static unsigned long long g_stat[20];
static unsigned long long g_mesh_tris[MAXM], g_mesh_nodes[MAXM], g_mesh_calls[MAXM], g_mesh_oct[MAXM], g_mesh_n[MAXM],
    g_mesh_steps[MAXM], g_mesh_skip[MAXM], g_mesh_skip1[MAXM], g_mesh_leafskip[MAXM], g_mesh_pair[MAXM];
enum { S_CALLS, S_REF_NODES, S_OCT_NODES, S_OCTM_NODES, S_STACK_BOX, S_STACK_POPS, S_OCT_MISMATCH, S_OCTM_MISMATCH,
       S_ANOM, S_TIE, S_STACK_MISMATCH, S_REF_HITS, S_REF_STEPS, S_CHAIN_STEPS, S_CHAIN_LEN, S_SKIP_STEPS, S_SKIP1_STEPS, S_LEAFSKIP_STEPS, S_MEAS_STEPS, S_PAIR_STEPS, S_NSTAT };

static void cen(const pt_bounding_box* b, float c[3]) {
    c[0] = 0.5f * (b->left_bottom.x + b->right_top.x);
    c[1] = 0.5f * (b->left_bottom.y + b->right_top.y);
    c[2] = 0.5f * (b->left_bottom.z + b->right_top.z);
}

static int emit(smesh* s, int k, int pos, int out, sn* arr) {
    const pt_bvh_node_device* nd = &s->ref[pos];
    sn* e = &arr[out];
    e->lo[0] = nd->box.left_bottom.x; e->lo[1] = nd->box.left_bottom.y; e->lo[2] = nd->box.left_bottom.z;
    e->hi[0] = nd->box.right_top.x; e->hi[1] = nd->box.right_top.y; e->hi[2] = nd->box.right_top.z;
    e->orig = pos;
    if (nd->is_leaf) {
        e->tri = nd->triangle_indices[0];
        e->skip = out + 1;
        return out + 1;
    }
    e->tri = -1;
    int l = s->left[pos], r = s->right[pos];
    float cl[3], cr[3];
    cen(&s->ref[l].box, cl);
    cen(&s->ref[r].box, cr);
    int ax = 0;
    float best = -1.0f;
    for (int a = 0; a < 3; a++) {
        float dd = fabsf(cl[a] - cr[a]);
        if (dd > best) { best = dd; ax = a; }
    }
    int neg = (k >> ax) & 1;  /* ray direction negative on the axis: visit the higher child first */
    int first = l, second = r;
    if ((cl[ax] > cr[ax]) != neg) { first = r; second = l; }
    int nx = emit(s, k, first, out + 1, arr);
    nx = emit(s, k, second, nx, arr);
    e->skip = nx;
    return nx;
}

static void prepare(const or_scene* sc, int m) {
    smesh* s = &g_mesh[m];
    if (s->n) return;
    const pt_bvh_node_device* nodes = sc->bvh[m];
    int n = nodes[0].next_node_index;
    s->ref = nodes;
    s->left = malloc(sizeof(int) * n);
    s->right = malloc(sizeof(int) * n);
    s->visits = calloc(n, sizeof(unsigned long long));
    s->passes = calloc(n, sizeof(unsigned long long));
    for (int p = 0; p < n; p++) {
        if (nodes[p].is_leaf) { s->left[p] = s->right[p] = -1; continue; }
        s->left[p] = p + 1;
        s->right[p] = nodes[p + 1].next_node_index;
    }
    for (int k = 0; k < 8; k++) {
        s->oct[k] = malloc(sizeof(sn) * n);
        int e = emit(s, k, 0, 0, s->oct[k]);
        if (e != n) { fprintf(stderr, "emit %d != %d\n", e, n); abort(); }
    }
    __atomic_store_n(&s->n, n, __ATOMIC_RELEASE);
}

static int sbox(const float lo[3], const float hi[3], or_v3 o, or_v3 inv, float* entry) {
    float tx1 = (lo[0] - o.x) * inv.x, tx2 = (hi[0] - o.x) * inv.x;
    float ty1 = (lo[1] - o.y) * inv.y, ty2 = (hi[1] - o.y) * inv.y;
    float tz1 = (lo[2] - o.z) * inv.z, tz2 = (hi[2] - o.z) * inv.z;
    float t_max = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
    float t_min = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
    *entry = t_max;
    return t_max <= t_min && t_min > 0.0f;
}

typedef struct { float t; int tri, orig; } best_t;

static void candidate(const or_scene* sc, int tri, int orig, float entry, or_v3 o, or_v3 d, best_t* b,
                      unsigned long long* anom, unsigned long long* tie) {
    float t, t1, t2;
    if (!triangle_intersect(&sc->tris[tri], o, d, &t, &t1, &t2) || !(t > 0.0f)) return;
    if (entry > t) (*anom)++;
    if (t < b->t || (t == b->t && orig < b->orig)) {
        if (t == b->t) (*tie)++;
        b->t = t; b->tri = tri; b->orig = orig;
    }
}

static void walk_oct(const or_scene* sc, const smesh* s, int k, or_v3 o, or_v3 d, or_v3 inv, float margin, best_t* b,
                     unsigned long long* nodes, unsigned long long* anom, unsigned long long* tie) {
    const sn* a = s->oct[k];
    int pos = 0;
    b->t = INFINITY; b->tri = -1; b->orig = 0x7fffffff;
    while (pos != s->n) {
        const sn* e = &a[pos];
        float entry;
        (*nodes)++;
        if (sbox(e->lo, e->hi, o, inv, &entry) && entry <= b->t * margin) {
            if (e->tri >= 0) candidate(sc, e->tri, e->orig, entry, o, d, b, anom, tie);
            pos++;
        } else {
            pos = e->skip;
        }
    }
}

static void walk_stack(const or_scene* sc, const smesh* s, or_v3 o, or_v3 d, or_v3 inv, best_t* b,
                       unsigned long long* boxes, unsigned long long* pops) {
    int stk[256];
    float ent[256];
    int sp = 0;
    unsigned long long an = 0, ti = 0;
    b->t = INFINITY; b->tri = -1; b->orig = 0x7fffffff;
    const pt_bvh_node_device* nd = s->ref;
    float e0;
    (*boxes)++;
    float lo[3] = {nd[0].box.left_bottom.x, nd[0].box.left_bottom.y, nd[0].box.left_bottom.z};
    float hi[3] = {nd[0].box.right_top.x, nd[0].box.right_top.y, nd[0].box.right_top.z};
    if (!sbox(lo, hi, o, inv, &e0)) return;
    stk[sp] = 0; ent[sp] = e0; sp++;
    while (sp) {
        sp--;
        int p = stk[sp];
        if (ent[sp] > b->t) continue;
        (*pops)++;
        if (nd[p].is_leaf) {
            candidate(sc, nd[p].triangle_indices[0], p, ent[sp], o, d, b, &an, &ti);
            continue;
        }
        int c[2] = {s->left[p], s->right[p]};
        float ce[2];
        int h[2];
        for (int i = 0; i < 2; i++) {
            const pt_bounding_box* bb = &nd[c[i]].box;
            float l3[3] = {bb->left_bottom.x, bb->left_bottom.y, bb->left_bottom.z};
            float h3[3] = {bb->right_top.x, bb->right_top.y, bb->right_top.z};
            (*boxes)++;
            h[i] = sbox(l3, h3, o, inv, &ce[i]) && ce[i] <= b->t;
        }
        int nearf = (h[0] && h[1]) ? (ce[1] < ce[0]) : (h[1] ? 1 : 0);
        int farf = 1 - nearf;
        if (h[farf]) { stk[sp] = c[farf]; ent[sp] = ce[farf]; sp++; }
        if (h[nearf]) { stk[sp] = c[nearf]; ent[sp] = ce[nearf]; sp++; }
        if (sp > 250) abort();
    }
}

static int box_pass(const pt_bounding_box* bb, or_v3 o, or_v3 inv, float bt) {
    float lo[3] = {bb->left_bottom.x, bb->left_bottom.y, bb->left_bottom.z};
    float hi[3] = {bb->right_top.x, bb->right_top.y, bb->right_top.z};
    float e;
    return sbox(lo, hi, o, inv, &e) && e <= bt;
}

static void study_hook(const void* scv, int m, float ox, float oy, float oz, float dx, float dy, float dz, int hit,
                       float t, int tri) {
    const or_scene* sc = (const or_scene*)scv;
    if (m >= MAXM) return;
    smesh* s = &g_mesh[m];
    if (!__atomic_load_n(&s->n, __ATOMIC_ACQUIRE)) {
#pragma omp critical(study_prep)
        prepare(sc, m);
    }
    or_v3 o = v3(ox, oy, oz), d = v3(dx, dy, dz);
    or_v3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    int k = (d.x < 0.0f) | ((d.y < 0.0f) << 1) | ((d.z < 0.0f) << 2);
    unsigned long long loc[S_NSTAT] = {0};
    loc[S_CALLS] = 1;
    loc[S_REF_HITS] = hit ? 1 : 0;
    /* reference node count: the preorder walk again (cheap to recount here) */
    {
        best_t b;
        unsigned long long an = 0, ti = 0;
        const pt_bvh_node_device* nd = s->ref;
        int pos = 0;
        b.t = INFINITY; b.tri = -1; b.orig = 0x7fffffff;
        while (pos != s->n) {
            float lo[3] = {nd[pos].box.left_bottom.x, nd[pos].box.left_bottom.y, nd[pos].box.left_bottom.z};
            float hi[3] = {nd[pos].box.right_top.x, nd[pos].box.right_top.y, nd[pos].box.right_top.z};
            float e;
            loc[S_REF_NODES]++;
            __atomic_fetch_add(&s->visits[pos], 1, __ATOMIC_RELAXED);
            if (sbox(lo, hi, o, inv, &e) && e <= b.t) {
                __atomic_fetch_add(&s->passes[pos], 1, __ATOMIC_RELAXED);
                if (nd[pos].is_leaf) {
                    float tt, t1, t2;
                    __atomic_fetch_add(&g_mesh_tris[m], 1, __ATOMIC_RELAXED);
                    int ti2 = nd[pos].triangle_indices[0];
                    if (triangle_intersect(&sc->tris[ti2], o, d, &tt, &t1, &t2) && tt > 0.0f && tt < b.t) {
                        b.t = tt; b.tri = ti2;
                    }
                }
                pos++;
            } else pos = nd[pos].next_node_index;
        }
        (void)an; (void)ti;
    }
    /* the GPU walk's dependent steps over the same preorder walk (pass_kernel_u, walk_box_inline): a step loads the
       records at pos and pos + 1; a passing internal node tests pos + 1 in the same step (a passing internal second
       record moves the walk to pos + 2, a passing leaf second record is re-tested with its triangle next step); a
       passing first-record leaf is tested with its triangle and the walk moves to pos + 1 */
    {
        const pt_bvh_node_device* nd = s->ref;
        float bt = INFINITY;
        int pos = 0;
        while (pos != s->n) {
            loc[S_REF_STEPS]++;
            float lo[3] = {nd[pos].box.left_bottom.x, nd[pos].box.left_bottom.y, nd[pos].box.left_bottom.z};
            float hi[3] = {nd[pos].box.right_top.x, nd[pos].box.right_top.y, nd[pos].box.right_top.z};
            float e;
            if (!(sbox(lo, hi, o, inv, &e) && e <= bt)) { pos = nd[pos].next_node_index; continue; }
            if (nd[pos].is_leaf) {
                float tt, t1, t2;
                int ti2 = nd[pos].triangle_indices[0];
                if (triangle_intersect(&sc->tris[ti2], o, d, &tt, &t1, &t2) && tt > 0.0f && tt < bt) bt = tt;
                pos++;
                continue;
            }
            const int q = pos + 1;
            float lo2[3] = {nd[q].box.left_bottom.x, nd[q].box.left_bottom.y, nd[q].box.left_bottom.z};
            float hi2[3] = {nd[q].box.right_top.x, nd[q].box.right_top.y, nd[q].box.right_top.z};
            if (!(sbox(lo2, hi2, o, inv, &e) && e <= bt)) pos = nd[q].next_node_index;
            else pos = nd[q].is_leaf ? q : q + 1;
        }
    }
    /* the same steps when the walk first skips the preorder chain root, root + 1, ... of internal nodes whose boxes
       hold the ray origin strictly inside (every such box passes: entry <= 0 < exit, and min_t is +inf at a mesh
       walk's start), at most CHAIN nodes; the root's own test is the segment start's (not counted as a step) */
    {
        const int CHAIN = 4;
        const pt_bvh_node_device* nd = s->ref;
        int pos = 0, len = 0;
        while (len < CHAIN && pos < s->n && !nd[pos].is_leaf) {
            const pt_bounding_box* bb = &nd[pos].box;
            if (!(bb->left_bottom.x < ox && ox < bb->right_top.x && bb->left_bottom.y < oy && oy < bb->right_top.y &&
                  bb->left_bottom.z < oz && oz < bb->right_top.z))
                break;
            pos++;
            len++;
        }
        loc[S_CHAIN_LEN] += len;
        float bt = INFINITY;
        while (pos != s->n) {
            loc[S_CHAIN_STEPS]++;
            float lo[3] = {nd[pos].box.left_bottom.x, nd[pos].box.left_bottom.y, nd[pos].box.left_bottom.z};
            float hi[3] = {nd[pos].box.right_top.x, nd[pos].box.right_top.y, nd[pos].box.right_top.z};
            float e;
            if (!(sbox(lo, hi, o, inv, &e) && e <= bt)) { pos = nd[pos].next_node_index; continue; }
            if (nd[pos].is_leaf) {
                float tt, t1, t2;
                int ti2 = nd[pos].triangle_indices[0];
                if (triangle_intersect(&sc->tris[ti2], o, d, &tt, &t1, &t2) && tt > 0.0f && tt < bt) bt = tt;
                pos++;
                continue;
            }
            const int q = pos + 1;
            float lo2[3] = {nd[q].box.left_bottom.x, nd[q].box.left_bottom.y, nd[q].box.left_bottom.z};
            float hi2[3] = {nd[q].box.right_top.x, nd[q].box.right_top.y, nd[q].box.right_top.z};
            if (!(sbox(lo2, hi2, o, inv, &e) && e <= bt)) pos = nd[q].next_node_index;
            else pos = nd[q].is_leaf ? q : q + 1;
        }
    }
    /* skip speculation: every record also carries the box of its skip target (and that target's own skip index), so
       a step at pos tests pos; when pos fails, skip(pos) in the same step; when pos passes (internal), pos + 1 and, if
       that fails, skip(pos + 1) (carried by pos + 1's record). The same visits in the same order as the reference's
       walk; a passing leaf met as a speculated record is re-tested with its triangle next step. */
    {
        const pt_bvh_node_device* nd = s->ref;
        float bt = INFINITY;
        int pos = 0;
#define PASSES(i) ((i) < s->n && box_pass(&nd[i].box, o, inv, bt))
        while (pos != s->n) {
            loc[S_SKIP_STEPS]++;
            if (!PASSES(pos)) {
                const int sk = nd[pos].next_node_index;
                if (sk == s->n) { pos = sk; continue; }
                if (PASSES(sk)) pos = nd[sk].is_leaf ? sk : sk + 1;
                else pos = nd[sk].next_node_index;
                continue;
            }
            if (nd[pos].is_leaf) {
                float tt, t1, t2;
                int ti2 = nd[pos].triangle_indices[0];
                if (triangle_intersect(&sc->tris[ti2], o, d, &tt, &t1, &t2) && tt > 0.0f && tt < bt) bt = tt;
                pos++;
                continue;
            }
            const int q = pos + 1;
            if (PASSES(q)) { pos = nd[q].is_leaf ? q : q + 1; continue; }
            const int sk = nd[q].next_node_index;
            if (sk == s->n) { pos = sk; continue; }
            if (PASSES(sk)) pos = nd[sk].is_leaf ? sk : sk + 1;
            else pos = nd[sk].next_node_index;
        }
        /* skip1: the same without skip(pos + 1): a failing pos + 1 moves the walk to its skip target untested (one
           speculated box per step: pos + 1's when pos passes, skip(pos)'s when it fails) */
        bt = INFINITY;
        pos = 0;
        while (pos != s->n) {
            loc[S_SKIP1_STEPS]++;
            if (!PASSES(pos)) {
                const int sk = nd[pos].next_node_index;
                if (sk == s->n) { pos = sk; continue; }
                if (PASSES(sk)) pos = nd[sk].is_leaf ? sk : sk + 1;
                else pos = nd[sk].next_node_index;
                continue;
            }
            if (nd[pos].is_leaf) {
                float tt, t1, t2;
                int ti2 = nd[pos].triangle_indices[0];
                if (triangle_intersect(&sc->tris[ti2], o, d, &tt, &t1, &t2) && tt > 0.0f && tt < bt) bt = tt;
                pos++;
                continue;
            }
            const int q = pos + 1;
            if (PASSES(q)) pos = nd[q].is_leaf ? q : q + 1;
            else pos = nd[q].next_node_index;
        }
        /* leafskip: the present layout (a leaf's skip target is the record after its triangle) with 96 B per step: a
           failing leaf's successor is tested in the same step; nothing else changes */
        bt = INFINITY;
        pos = 0;
        while (pos != s->n) {
            loc[S_LEAFSKIP_STEPS]++;
            if (!PASSES(pos)) {
                const int sk = nd[pos].next_node_index;
                if (!nd[pos].is_leaf || sk == s->n) { pos = sk; continue; }
                if (PASSES(sk)) pos = nd[sk].is_leaf ? sk : sk + 1;
                else pos = nd[sk].next_node_index;
                continue;
            }
            if (nd[pos].is_leaf) {
                float tt, t1, t2;
                int ti2 = nd[pos].triangle_indices[0];
                if (triangle_intersect(&sc->tris[ti2], o, d, &tt, &t1, &t2) && tt > 0.0f && tt < bt) bt = tt;
                pos++;
                continue;
            }
            const int q = pos + 1;
            if (PASSES(q)) pos = nd[q].is_leaf ? q : q + 1;
            else pos = nd[q].next_node_index;
        }
#undef PASSES
    }
    /* pair merge: an internal node P whose children are two leaves, the first with P's own box (bit for bit: a thin
       leaf widened to its parent's), is dropped from the layout; its first leaf carries P's test (same box, same
       min_t) and a failing test skips both leaves. The GPU two-record step otherwise as ref_steps. */
    {
        const pt_bvh_node_device* nd = s->ref;
#define MERGED(i) ((i) + 2 < s->n && !nd[i].is_leaf && nd[(i) + 1].is_leaf && nd[(i) + 2].is_leaf && \
                   nd[i].next_node_index == (i) + 3 && !memcmp(&nd[i].box, &nd[(i) + 1].box, sizeof(pt_bounding_box)))
        float bt = INFINITY;
        int pos = 0;
        while (pos != s->n) {
            loc[S_PAIR_STEPS]++;
            float e;
            if (MERGED(pos)) pos++;  /* the walk stands on the merged leaf (P's record does not exist) */
            if (!box_pass(&nd[pos].box, o, inv, bt)) {
                pos = (pos > 0 && nd[pos].is_leaf && MERGED(pos - 1)) ? pos + 2 : nd[pos].next_node_index;
                continue;
            }
            if (nd[pos].is_leaf) {
                float tt, t1, t2;
                int ti2 = nd[pos].triangle_indices[0];
                if (triangle_intersect(&sc->tris[ti2], o, d, &tt, &t1, &t2) && tt > 0.0f && tt < bt) bt = tt;
                pos++;
                continue;
            }
            int q = pos + 1;
            int qm = MERGED(q);
            if (qm) q++;
            if (!box_pass(&nd[q].box, o, inv, bt)) pos = qm ? q + 2 : nd[q].next_node_index;
            else pos = nd[q].is_leaf ? q : q + 1;
            (void)e;
        }
#undef MERGED
    }
    if (s->meas) {  /* the GPU two-record step over the measured-order copy (study_reorder) */
        const sn* a = s->meas;
        float bt = INFINITY, e;
        int pos = 0;
        while (pos != s->n) {
            loc[S_MEAS_STEPS]++;
            if (!(sbox(a[pos].lo, a[pos].hi, o, inv, &e) && e <= bt)) { pos = a[pos].skip; continue; }
            if (a[pos].tri >= 0) {
                float tt, t1, t2;
                if (triangle_intersect(&sc->tris[a[pos].tri], o, d, &tt, &t1, &t2) && tt > 0.0f && tt < bt) bt = tt;
                pos++;
                continue;
            }
            const int q = pos + 1;
            if (!(sbox(a[q].lo, a[q].hi, o, inv, &e) && e <= bt)) pos = a[q].skip;
            else pos = a[q].tri >= 0 ? q : q + 1;
        }
    }
    best_t b;
    walk_oct(sc, s, k, o, d, inv, 1.0f, &b, &loc[S_OCT_NODES], &loc[S_ANOM], &loc[S_TIE]);
    int same = hit ? (b.tri == tri && b.t == t) : (b.tri < 0);
    if (!same) loc[S_OCT_MISMATCH]++;
    unsigned long long dummy = 0;
    walk_oct(sc, s, k, o, d, inv, 1.0f + 1.0f / 1024.0f, &b, &loc[S_OCTM_NODES], &dummy, &dummy);
    same = hit ? (b.tri == tri && b.t == t) : (b.tri < 0);
    if (!same) loc[S_OCTM_MISMATCH]++;
    walk_stack(sc, s, o, d, inv, &b, &loc[S_STACK_BOX], &loc[S_STACK_POPS]);
    same = hit ? (b.tri == tri && b.t == t) : (b.tri < 0);
    if (!same) loc[S_STACK_MISMATCH]++;
    for (int i = 0; i < S_NSTAT; i++) __atomic_fetch_add(&g_stat[i], loc[i], __ATOMIC_RELAXED);
    __atomic_fetch_add(&g_mesh_nodes[m], loc[S_REF_NODES], __ATOMIC_RELAXED);
    __atomic_fetch_add(&g_mesh_oct[m], loc[S_OCT_NODES], __ATOMIC_RELAXED);
    __atomic_fetch_add(&g_mesh_steps[m], loc[S_REF_STEPS], __ATOMIC_RELAXED);
    __atomic_fetch_add(&g_mesh_skip[m], loc[S_SKIP_STEPS], __ATOMIC_RELAXED);
    __atomic_fetch_add(&g_mesh_skip1[m], loc[S_SKIP1_STEPS], __ATOMIC_RELAXED);
    __atomic_fetch_add(&g_mesh_leafskip[m], loc[S_LEAFSKIP_STEPS], __ATOMIC_RELAXED);
    __atomic_fetch_add(&g_mesh_pair[m], loc[S_PAIR_STEPS], __ATOMIC_RELAXED);
    __atomic_fetch_add(&g_mesh_calls[m], 1, __ATOMIC_RELAXED);
    g_mesh_n[m] = s->n;
}


static double sa(const pt_bounding_box* b) {
    double x = b->right_top.x - b->left_bottom.x, y = b->right_top.y - b->left_bottom.y, z = b->right_top.z - b->left_bottom.z;
    return x * y + y * z + z * x;
}
/* share of visits landing on a top tree of `budget` nodes: BFS levels, or greedy by surface area */
static void coverage(smesh* s, int budget) {
    int n = s->n;
    unsigned long long tot = 0;
    for (int p = 0; p < n; p++) tot += s->visits[p];
    char* in = calloc(n, 1);
    int cnt = 1;
    in[0] = 1;
    /* greedy: repeatedly expand the top-leaf internal node of largest surface area */
    while (cnt + 2 <= budget) {
        int bestp = -1; double bs = -1;
        for (int p = 0; p < n; p++)
            if (in[p] && s->left[p] >= 0 && !in[s->left[p]]) { double a = sa(&s->ref[p].box); if (a > bs) { bs = a; bestp = p; } }
        if (bestp < 0) break;
        in[s->left[bestp]] = in[s->right[bestp]] = 1; cnt += 2;
    }
    unsigned long long cov = 0;
    for (int p = 0; p < n; p++) if (in[p]) cov += s->visits[p];
    /* BFS */
    char* in2 = calloc(n, 1);
    int* q = malloc(sizeof(int) * n); int qh = 0, qt = 0, c2 = 1; q[qt++] = 0; in2[0] = 1;
    while (qh < qt) { int p = q[qh++]; if (s->left[p] < 0) continue; if (c2 + 2 > budget) break;
        in2[s->left[p]] = in2[s->right[p]] = 1; c2 += 2; q[qt++] = s->left[p]; q[qt++] = s->right[p]; }
    unsigned long long cov2 = 0;
    for (int p = 0; p < n; p++) if (in2[p]) cov2 += s->visits[p];
    printf("    budget %5d: SA-greedy %d nodes cover %.3f of visits; BFS %d nodes cover %.3f\n", budget, cnt,
           (double)cov / tot, c2, (double)cov2 / tot);
    free(in); free(in2); free(q);
}

/* study_reorder: each mesh's children re-ordered by the expected GPU steps (pt_sah_order_by_steps' recurrence) under the
   MEASURED pass probabilities of the sample rendered so far (passes[child] / passes[parent]), into s->meas; the next
   render's walks are counted over it (S_MEAS_STEPS). mode 1: measured probabilities, 0: the surface-area ratio
   (the shipped order 6 recomputed, a check). */
static double *g_start, *g_free;
static double sa(const pt_bounding_box* b);
/* start(Y) = 1 + P(Y)(free(F) + start(S)), free(Y) = P(Y)(start(F) + start(S)); leaf: start 1, free P */
static void dp(smesh* s, int p, double P, int mode) {
    if (s->left[p] < 0) { g_start[p] = 1.0; g_free[p] = P; return; }
    int c[2] = {s->left[p], s->right[p]};
    for (int i = 0; i < 2; i++) {
        double pr;
        if (mode == 1) pr = s->passes[p] ? (double)s->passes[c[i]] / (double)s->passes[p] : 0.0;
        else {
            const pt_bounding_box* cb = &s->ref[c[i]].box;
            int thin = cb->left_bottom.x == cb->right_top.x || cb->left_bottom.y == cb->right_top.y ||
                       cb->left_bottom.z == cb->right_top.z;
            double sp = sa(&s->ref[p].box);
            pr = (s->left[c[i]] < 0 && thin) || !(sp > 0.0) ? 1.0 : fmin(1.0, sa(cb) / sp);
        }
        dp(s, c[i], pr > 1.0 ? 1.0 : pr, mode);
    }
    double a = g_free[c[0]] + g_start[c[1]], b = g_free[c[1]] + g_start[c[0]];
    if (b < a) { s->left[p] = c[1]; s->right[p] = c[0]; a = b; }
    g_start[p] = 1.0 + P * a;
    g_free[p] = P * (g_start[c[0]] + g_start[c[1]]);
}
static int emit_meas(smesh* s, int p, int out) {
    const pt_bvh_node_device* nd = &s->ref[p];
    sn* e = &s->meas[out];
    e->lo[0] = nd->box.left_bottom.x; e->lo[1] = nd->box.left_bottom.y; e->lo[2] = nd->box.left_bottom.z;
    e->hi[0] = nd->box.right_top.x; e->hi[1] = nd->box.right_top.y; e->hi[2] = nd->box.right_top.z;
    e->orig = p;
    if (s->left[p] < 0) { e->tri = nd->triangle_indices[0]; e->skip = out + 1; return out + 1; }
    e->tri = -1;
    int nx = emit_meas(s, s->left[p], out + 1);
    nx = emit_meas(s, s->right[p], nx);
    e->skip = nx;
    return nx;
}
void study_reorder(int mode) {
    for (int m = 0; m < MAXM; m++) {
        smesh* s = &g_mesh[m];
        if (!s->n) continue;
        g_start = calloc(s->n, sizeof(double));
        g_free = calloc(s->n, sizeof(double));
        dp(s, 0, 1.0, mode);
        s->meas = malloc(sizeof(sn) * s->n);
        if (emit_meas(s, 0, 0) != s->n) abort();
        free(g_start); free(g_free);
    }
}

void study_stats(unsigned long long* out) {
    for (int m = 0; m < MAXM; m++)
        if (g_mesh[m].n > 1000) { int b[] = {64, 128, 256, 512, 1024, 2048, 4096}; for (int i = 0; i < 7; i++) coverage(&g_mesh[m], b[i]); }
    for (int i = 0; i < S_NSTAT; i++) out[i] = g_stat[i];
    for (int m = 0; m < MAXM; m++)
        if (g_mesh_calls[m])
            printf("  mesh %d: %llu nodes, %llu walks, ref nodes/walk %.2f, steps/walk %.2f, skip-spec steps/walk %.2f (one box: %.2f, leaves only: %.2f), pair-merged steps/walk %.2f, "
                   "tris/walk %.2f, oct nodes/walk %.2f\n",
                   m, g_mesh_n[m], g_mesh_calls[m], (double)g_mesh_nodes[m] / g_mesh_calls[m],
                   (double)g_mesh_steps[m] / g_mesh_calls[m], (double)g_mesh_skip[m] / g_mesh_calls[m],
                   (double)g_mesh_skip1[m] / g_mesh_calls[m], (double)g_mesh_leafskip[m] / g_mesh_calls[m],
                   (double)g_mesh_pair[m] / g_mesh_calls[m],
                   (double)g_mesh_tris[m] / g_mesh_calls[m],
                   (double)g_mesh_oct[m] / g_mesh_calls[m]);
    fflush(stdout);
}
