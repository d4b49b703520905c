/*
 * leaf_position_study.c — STUDY TOOL (test infrastructure, never linked into the product).
 *
 * Replays every mesh walk of the oracle (oracle.c mesh_bvh, path_tracer_kernel.cu:111-150) with the
 * GPU walk's step boundaries (pt_path.h walk_box_chain<2>: a step tests record pos and, after a
 * passing internal record, pos + 1; a passing leaf ends the step) and counts, for every leaf whose box
 * passes, whether it was the step's first or second record. A layout that stores a leaf's triangle
 * in the 32 B after its box record would have the triangle in registers for first-record leaves.
 *
 *   python tools/leaf_position_study.py [sample]
 */
#include <stdint.h>
#include <stdio.h>

static void study_hook(const void* sc, int m, float ox, float oy, float oz, float dx, float dy, float dz, int hit,
                       float t, int tri);
#define OR_STUDY_HOOK(sc, m, o, d, hit, t, tri) study_hook(sc, m, o.x, o.y, o.z, d.x, d.y, d.z, hit, t, tri)
#include "../oracle/oracle.c"

enum { S_WALKS, S_STEPS, S_LEAF1, S_LEAF2, S_REC, S_MISMATCH, S_N };
static unsigned long long g_stat[S_N];

static void study_hook(const void* scv, int m, float ox, float oy, float oz, float dx, float dy, float dz, int hit,
                       float t_ref, int tri_ref) {
    const or_scene* sc = (const or_scene*)scv;
    or_v3 o = v3(ox, oy, oz), d = v3(dx, dy, dz);
    const pt_bvh_node_device* nodes = sc->bvh[m];
    const int n = nodes[0].next_node_index;
    float min_t = INFINITY, box_t = INFINITY;
    int min_tri = -1;
    unsigned long long st[S_N] = {0};
    st[S_WALKS] = 1;
    int pos = 0;
    while (pos != n) {
        st[S_STEPS]++;
        for (int k = 0; k < 2 && pos != n; k++) {
            const pt_bvh_node_device* nd = &nodes[pos];
            st[S_REC]++;
            if (box_intersect(&nd->box, o, d, &box_t) && box_t <= min_t) {
                if (nd->is_leaf) {
                    st[k == 0 ? S_LEAF1 : S_LEAF2]++;
                    int ti = nd->triangle_indices[0];
                    float t, t1, t2;
                    if (ti >= 0 && triangle_intersect(&sc->tris[ti], o, d, &t, &t1, &t2) && t > 0.0f && t < min_t) {
                        min_t = t; min_tri = ti;
                    }
                    pos++;
                    break;  /* a passing leaf ends the step */
                }
                pos++;
            } else {
                pos = nd->next_node_index;
                break;
            }
        }
    }
    if ((hit ? min_tri : -1) != (hit ? tri_ref : -1)) st[S_MISMATCH]++;
#pragma omp critical
    for (int i = 0; i < S_N; i++) g_stat[i] += st[i];
}

void study_stats(unsigned long long* out) {
    for (int i = 0; i < S_N; i++) out[i] = g_stat[i];
}
