/*
 * layout_study.c — STUDY TOOL (test infrastructure, never linked into the product).
 *
 * Replays every mesh walk of the oracle (oracle.c mesh_bvh, path_tracer_kernel.cu:85-161) and counts, for
 * the SAME visit sequence (the reference's preorder walk with its min_t), the dependent record loads
 * ("steps") two record layouts would need:
 *   chain2   — the product's walk step (pt_path.h walk_box_chain<2>): a step loads the node at pos and the
 *              next record in preorder; a passing internal node's left child is tested from the same
 *              load; a passing leaf ends the step (its triangle is tested, the walk resumes at pos + 1).
 *   children — a parent record holding both children's boxes: at a passing internal node p, one load
 *              gives box(left) and box(right); a failing left child lets the right one be tested from the
 *              same load; a passing internal child is the next load; after a leaf the walk reloads the
 *              parent for the right child (reload_after_leaf) or keeps it (kept); after a right subtree the
 *              walk loads the record holding the skip target's box (its parent).
 * Both visit exactly the reference's nodes in the same order (the records only move boxes around).
 *
 *   python tools/layout_study.py [pixels] [passes]
 */
#include <stdint.h>
#include <stdio.h>

static void study_hook(const void* sc, int m, float ox, float oy, float oz, float dx, float dy, float dz, int hit,
                       float t, int tri);
#define OR_STUDY_HOOK(sc, m, o, d, hit, t, tri) study_hook(sc, m, o.x, o.y, o.z, d.x, d.y, d.z, hit, t, tri)
#include "../oracle/oracle.c"

enum { L_CALLS, L_VISITS, L_CHAIN2, L_CHILD_RELOAD, L_CHILD_KEPT, L_TRIS, L_N };
static unsigned long long g_l[L_N];
#define MAXM 16
static unsigned long long g_mesh[MAXM][L_N];

/* parent of every node and whether it is a left child, per mesh (built once) */
typedef struct { int n; int* parent; unsigned char* is_left; } lmesh;
static lmesh g_lm[MAXM];

static void lprepare(const pt_bvh_node_device* nd, lmesh* s) {
    int n = nd[0].next_node_index;
    s->parent = malloc(sizeof(int) * n);
    s->is_left = malloc(n);
    s->parent[0] = -1; s->is_left[0] = 0;
    for (int p = 0; p < n; p++) {
        if (nd[p].is_leaf) continue;
        int l = p + 1, r = nd[p + 1].next_node_index;
        s->parent[l] = p; s->is_left[l] = 1;
        if (r < nd[p].next_node_index) { s->parent[r] = p; s->is_left[r] = 0; }
    }
    __atomic_store_n(&s->n, n, __ATOMIC_RELEASE);
}

static int lbox(const pt_bvh_node_device* nd, int p, or_v3 o, or_v3 inv, float* entry) {
    const pt_bounding_box* b = &nd[p].box;
    float tx1 = (b->left_bottom.x - o.x) * inv.x, tx2 = (b->right_top.x - o.x) * inv.x;
    float ty1 = (b->left_bottom.y - o.y) * inv.y, ty2 = (b->right_top.y - o.y) * inv.y;
    float tz1 = (b->left_bottom.z - o.z) * inv.z, tz2 = (b->right_top.z - o.z) * inv.z;
    float t_max = fmaxf(fmaxf(fminf(tx1, tx2), fminf(ty1, ty2)), fminf(tz1, tz2));
    float t_min = fminf(fminf(fmaxf(tx1, tx2), fmaxf(ty1, ty2)), fmaxf(tz1, tz2));
    *entry = t_max;
    return t_max <= t_min && t_min > 0.0f;
}

static void study_hook(const void* scv, int m, float ox, float oy, float oz, float dx, float dy, float dz, int hit,
                       float t, int tri) {
    (void)hit; (void)t; (void)tri;
    const or_scene* sc = (const or_scene*)scv;
    if (m >= MAXM) return;
    const pt_bvh_node_device* nd = sc->bvh[m];
    lmesh* s = &g_lm[m];
    if (!__atomic_load_n(&s->n, __ATOMIC_ACQUIRE)) {
#pragma omp critical(layout_prep)
        if (!s->n) lprepare(nd, s);
    }
    const int n = s->n;
    or_v3 o = v3(ox, oy, oz), d = v3(dx, dy, dz);
    or_v3 inv = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    unsigned long long c[L_N] = {0};
    c[L_CALLS] = 1;
    /* the reference walk, recording each visited node's outcome: 0 fail, 1 pass internal, 2 pass leaf */
    int seq_node[4096];
    unsigned char seq_out[4096];
    int k = 0;
    float min_t = INFINITY;
    int pos = 0;
    while (pos != n) {
        float e;
        int pass = lbox(nd, pos, o, inv, &e) && e <= min_t;
        if (k < 4096) { seq_node[k] = pos; seq_out[k] = pass ? (nd[pos].is_leaf ? 2 : 1) : 0; }
        k++;
        if (pass) {
            if (nd[pos].is_leaf) {
                float tt, t1, t2;
                c[L_TRIS]++;
                if (triangle_intersect(&sc->tris[nd[pos].triangle_indices[0]], o, d, &tt, &t1, &t2) && tt > 0.0f &&
                    tt < min_t)
                    min_t = tt;
            }
            pos++;
        } else pos = nd[pos].next_node_index;
    }
    if (k > 4096) return; /* not expected for these scenes */
    c[L_VISITS] = (unsigned long long)k;
    /* chain2: a step covers visit i, and visit i + 1 when visit i passed an internal node (its left child) */
    for (int i = 0; i < k;) {
        c[L_CHAIN2]++;
        if (seq_out[i] == 1 && i + 1 < k) {
            i += 2;
        } else {
            i += 1;
        }
    }
    /* children layout: visiting node v needs the record of parent(v) in registers (the root: one load).
       In registers after a step: the record of the last internal node whose children were tested. */
    for (int variant = 0; variant < 2; variant++) {
        unsigned long long loads = 0;
        int have = -2; /* record held: parent index, -2 none (the root record counts as parent -1) */
        for (int i = 0; i < k; i++) {
            int v = seq_node[i];
            int p = s->parent[v];
            if (have != p) { loads++; have = p; }
            if (seq_out[i] == 2 && variant == 0) have = -2; /* parked on a leaf: registers reused */
            /* a passing internal node: its children are tested next, from its own record (loaded when needed) */
        }
        c[variant == 0 ? L_CHILD_RELOAD : L_CHILD_KEPT] = loads;
    }
    for (int i = 0; i < L_N; i++) {
        __atomic_fetch_add(&g_l[i], c[i], __ATOMIC_RELAXED);
        __atomic_fetch_add(&g_mesh[m][i], c[i], __ATOMIC_RELAXED);
    }
}

void layout_stats(unsigned long long* out, unsigned long long* per_mesh) {
    for (int i = 0; i < L_N; i++) out[i] = g_l[i];
    for (int m = 0; m < MAXM; m++)
        for (int i = 0; i < L_N; i++) per_mesh[m * L_N + i] = g_mesh[m][i];
}
