// pt_bvh_internal.h — the hand-off between the Morton builders' first half (host: pt_host.cpp,
// device: pt_bvh.hip) and their shared second half (pt_morton_finish in pt_host.cpp).
#pragma once

#include <vector>

#include "../../include/pt_types.h"
#include "pt_bvh_common.h"

// Sorted leaves and the Karras internal nodes of one mesh (Bvh/bvh.cpp:862-972).
struct PtMortonTree {
    unsigned int leaf_num = 0, internal_num = 0;
    std::vector<ptbvh::Box> leaf_box;  // leaves in Morton order
    std::vector<int> leaf_batch;       // batch of each sorted leaf (index into batch_tris / leaf_size)
    std::vector<int> batch_tris;       // leaf_num * leaf_size triangle ids, -1 padded
    std::vector<int> inner_left, inner_right;  // child: >= 0 internal id, <= -2 leaf -(id + 2)
    std::vector<int> inner_parent, leaf_parent;  // -1 = none
};

// leaf count of bvh.cpp:866-868. With fewer triangles than a leaf holds the reference's formula gives
// two leaves, and the second one's first triangle is read past the end of the sorted array (:926-933,
// undefined; found by the sanitizer build, tests/test_sanitizers.py): here that mesh is one leaf.
inline unsigned int pt_leaf_count(int n, int leaf_size) {
    if (n < leaf_size) return 1;
    unsigned int l = (unsigned int)(n / leaf_size);
    l = l == 0 ? 1 : l;
    return (n % leaf_size == 0) ? l : l + 1;
}

// Bottom-up boxes and the flattened skip-pointer array (Bvh/bvh.cpp:974-1047, :244-330).
int pt_morton_finish(PtMortonTree& t, int leaf_size, pt_bvh_node_device** nodes_out, int* node_num_out,
                     int** leaf_out, int* leaf_num_out);

// A linked tree (bvh_naive_cpu's build nodes, PT_BVH_SAH's, host or device): node 0 is the root; a leaf holds
// leaf_size triangle ids (-1 padded).
struct PtTreeNode {
    ptbvh::Box box;
    int left = -1, right = -1, parent = -1;
    bool leaf = false;
    std::vector<int> tris;
};

// build_bvh_device_data (Bvh/bvh.cpp:244-330) over a linked tree: preorder, skip indices, thin leaf boxes widened to
// the parent's (pt_host.cpp).
int pt_flatten_tree(std::vector<PtTreeNode>& nodes, int leaf_size, pt_bvh_node_device** nodes_out, int* node_num_out,
                    int** leaf_out, int* leaf_num_out);

// PT_BVH_SAH's preorder child order (PT_SAH_ORDER, pt_host.cpp) and order 6's bottom-up reordering of a built tree by
// the walk's expected dependent steps (both builders apply it before flattening).
int pt_sah_order();
int pt_sah_bins();
void pt_sah_order_by_steps(std::vector<PtTreeNode>& nodes);
// the tree study's treelet restructuring (pt_host.cpp; PT_SAH_TREELET / PT_LBVH_TREELET)
void pt_treelet_restructure(std::vector<PtTreeNode>& nodes, int k);
