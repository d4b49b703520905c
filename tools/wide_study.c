/*
 * wide_study.c — STUDY TOOL (test infrastructure, never linked into the product).
 *
 * Replays every mesh walk of the oracle (hook in oracle.c mesh_bvh, path_tracer_kernel.cu:85-161)
 * through stackless WIDE walks over collapsed copies of the same binary BVH, children kept in the
 * binary preorder, and counts what they cost against the binary walk the GPU runs today (two records
 * per step, pass_kernel_u CHAIN=2):
 *   wide    — a wide node = a binary internal node's children, each internal child replaced by ITS
 *             children (2-level collapse, 2-4 children), or greedily expanded by box area up to W
 *             children; slots tested in order with the running min_t; an internal slot that passes is
 *             descended (its wide record is the next step), a leaf slot that passes has its triangle
 *             tested, then the scan goes on at the next slot (same record kept, or reloaded).
 * Closest hits must equal the reference's (same leaves, same order, same min_t): checked per walk.
 *
 *   python tools/wide_study.py [PIXELS]
 */
#include <stdint.h>
#include <stdio.h>

static void study_hook(const void* sc, int m, float ox, float oy, float oz, float dx, float dy, float dz, int hit,
                       float t, int tri);
#define OR_STUDY_HOOK(sc, m, o, d, hit, t, tri) study_hook(sc, m, o.x, o.y, o.z, d.x, d.y, d.z, hit, t, tri)
#include "../oracle/oracle.c"

#define MAXW 8
typedef struct { int n; int child[MAXW]; int ref[MAXW]; int skip_w, skip_k; } wnode;  /* ref: >=0 wide, <0 leaf -(bin+1) */
typedef struct { int built; int nb; const pt_bvh_node_device* b; int* left; int* right; wnode* w; int nw; int root; } wmesh;

#define MAXM 16
#define NV 3
static wmesh g_m[NV][MAXM];
static int g_width[NV] = {4, 4, 8};
static int g_greedy[NV] = {0, 1, 1};
static unsigned long long g_st[32];
enum { CALLS, BIN_NODES, BIN_STEPS, BIN_TRIS, W_STEPS0, W_STEPS_RELOAD0, W_BOX0, W_MISMATCH0 };
#define WS(v, k) (W_STEPS0 + 4 * (v) + (k))

static float area(const pt_bounding_box* b) {
    float x = b->right_top.x - b->left_bottom.x, y = b->right_top.y - b->left_bottom.y, z = b->right_top.z - b->left_bottom.z;
    return x * y + y * z + z * x;
}

static int build_w(wmesh* M, int v, int bin) {
    int id = M->nw++;
    wnode nd;
    memset(&nd, 0, sizeof(nd));
    int list[MAXW], n = 0;
    list[n++] = M->left[bin];
    list[n++] = M->right[bin];
    if (!g_greedy[v]) {
        int out[MAXW], m = 0;
        for (int i = 0; i < n; i++) {
            int c = list[i];
            if (M->b[c].is_leaf) out[m++] = c;
            else { out[m++] = M->left[c]; out[m++] = M->right[c]; }
        }
        memcpy(list, out, sizeof(int) * m);
        n = m;
    } else {
        while (n < g_width[v]) {
            int best = -1;
            float ba = -1.0f;
            for (int i = 0; i < n; i++)
                if (!M->b[list[i]].is_leaf && area(&M->b[list[i]].box) > ba) { ba = area(&M->b[list[i]].box); best = i; }
            if (best < 0) break;
            int c = list[best];
            for (int i = n; i > best + 1; i--) list[i] = list[i - 1];
            list[best] = M->left[c];
            list[best + 1] = M->right[c];
            n++;
        }
    }
    nd.n = n;
    for (int i = 0; i < n; i++) nd.child[i] = list[i];
    M->w[id] = nd;
    for (int i = 0; i < n; i++) {
        int c = list[i];
        M->w[id].ref[i] = M->b[c].is_leaf ? -(c + 1) : build_w(M, v, c);
    }
    return id;
}

static void set_skips(wmesh* M, int w, int sw, int sk) {
    M->w[w].skip_w = sw;
    M->w[w].skip_k = sk;
    for (int i = 0; i < M->w[w].n; i++) {
        int r = M->w[w].ref[i];
        if (r < 0) continue;
        if (i + 1 < M->w[w].n) set_skips(M, r, w, i + 1);
        else set_skips(M, r, sw, sk);
    }
}

static void prepare(const or_scene* sc, int m) {
    for (int v = 0; v < NV; v++) {
        wmesh* M = &g_m[v][m];
        if (M->built) continue;
        const pt_bvh_node_device* b = sc->bvh[m];
        int n = b[0].next_node_index;
        M->b = b;
        M->nb = n;
        M->left = malloc(sizeof(int) * n);
        M->right = malloc(sizeof(int) * n);
        for (int p = 0; p < n; p++) {
            M->left[p] = M->right[p] = -1;
            if (!b[p].is_leaf) { M->left[p] = p + 1; M->right[p] = b[p + 1].next_node_index; }
        }
        M->w = malloc(sizeof(wnode) * (n + 1));
        M->nw = 0;
        if (b[0].is_leaf) {  /* one-leaf mesh: a wide node with the root as its only slot */
            M->w[0].n = 1; M->w[0].child[0] = 0; M->w[0].ref[0] = -1; M->nw = 1;
        } else {
            build_w(M, v, 0);
        }
        set_skips(M, 0, -1, 0);
        M->built = 1;
    }
}

static int box_pass(const pt_bounding_box* bx, or_v3 o, or_v3 d, float min_t) {
    float e;
    return box_intersect(bx, o, d, &e) && e <= min_t;
}

static void tri_test(const or_scene* sc, int ti, or_v3 o, or_v3 d, float* mt, int* mtri) {
    float t, t1, t2;
    if (triangle_intersect(&sc->tris[ti], o, d, &t, &t1, &t2) && t > 0.0f && t < *mt) { *mt = t; *mtri = ti; }
}

static void study_hook(const void* scv, int m, float ox, float oy, float oz, float dx, float dy, float dz, int hit,
                       float t, int tri) {
    const or_scene* sc = (const or_scene*)scv;
    unsigned long long loc[32] = {0};
    #pragma omp critical
    prepare(sc, m);
    or_v3 o = v3(ox, oy, oz), d = v3(dx, dy, dz);
    const pt_bvh_node_device* b = sc->bvh[m];
    int n = b[0].next_node_index;
    loc[CALLS]++;
    /* binary walk, two records per step (pass_kernel_u CHAIN=2) */
    {
        float mt = INFINITY;
        int mtri = -1, pos = 0;
        while (pos != n) {
            loc[BIN_STEPS]++;
            for (int c = 0; c < 2 && pos != n; c++) {
                loc[BIN_NODES]++;
                if (box_pass(&b[pos].box, o, d, mt)) {
                    if (b[pos].is_leaf) { loc[BIN_TRIS]++; tri_test(sc, b[pos].triangle_indices[0], o, d, &mt, &mtri); pos++; break; }
                    pos++;
                } else { pos = b[pos].next_node_index; break; }
            }
        }
    }
    for (int v = 0; v < NV; v++) {
        wmesh* M = &g_m[v][m];
        float mt = INFINITY;
        int mtri = -1, w = 0, k = 0;
        while (w >= 0) {
            loc[WS(v, 0)]++;
            loc[WS(v, 1)]++;
            const wnode* nd = &M->w[w];
            int moved = 0;
            for (int j = k; j < nd->n; j++) {
                loc[WS(v, 2)]++;
                int c = nd->child[j];
                if (!box_pass(&b[c].box, o, d, mt)) continue;
                if (nd->ref[j] < 0) {
                    tri_test(sc, b[c].triangle_indices[0], o, d, &mt, &mtri);
                    if (j + 1 < nd->n) loc[WS(v, 1)]++;  /* the reload variant re-fetches the record */
                    continue;
                }
                w = nd->ref[j]; k = 0; moved = 1;
                break;
            }
            if (!moved) { k = nd->skip_k; w = nd->skip_w; }
        }
        int ok = (mtri == tri) && (mtri < 0 || mt == t);
        if (!ok) loc[WS(v, 3)]++;
    }
    (void)hit;
    for (int i = 0; i < 32; i++) {
        if (!loc[i]) continue;
        #pragma omp atomic
        g_st[i] += loc[i];
    }
}

void study_stats(unsigned long long* out) { memcpy(out, g_st, sizeof(g_st)); }
