/*
 * pt_bvh.h — the GPU BVH builder (row f1): the reference's MortonCodeCUDA build ABI, plus a native
 * whole-mesh build.
 *
 *   compute_triangle_bounding_box_kernel  <- Kernel/bvh_morton_code_kernel.cu:348-370 (declared in
 *                                            Bvh/bvh_morton_code_kernel.h:10-17)
 *   generate_internal_node_kernel         <- Kernel/bvh_morton_code_kernel.cu:372-392 (:19-25)
 *   radix_sort                            <- Kernel/parallel_function.cu:22-32 (Core/parallel_function.h:13-17)
 *   pt_bvh_build_device                   <- bvh_morton_code_cuda::build_bvh + build_bvh_device_data
 *                                            (Bvh/bvh.cpp:862-1047, :244-330)
 *
 * Pointers handed to the reference entry points may be device memory or ordinary host memory (the
 * reference's are cudaMallocManaged); host buffers are staged through HBM. Like the reference the
 * calls are synchronous and print "[Hip]Error ..." on failure. block_size is accepted for ABI
 * compatibility; the kernels run 256-lane workgroups (four 64-lane waves).
 *
 * Results equal the host builder's (pt_bvh_build) bit for bit: the same arithmetic
 * (pt_bvh_common.h), stable radix sorts (thrust::sort's merge sort is stable), and parent links
 * resolved to the largest writing node as the host's sequential loop resolves them.
 */
#ifndef PT_BVH_H
#define PT_BVH_H

#include "pt_types.h"

#ifdef __cplusplus
extern "C" {
#endif

void compute_triangle_bounding_box_kernel(pt_triangle* triangles_device, int triangle_num,
                                          pt_bvh_node_morton_code_cuda* triangle_nodes_device,
                                          pt_bounding_box* mesh_box, int start_index, int block_size);
void generate_internal_node_kernel(pt_bvh_node_morton_code_cuda* internal_nodes_device, unsigned int internal_node_num,
                                   pt_bvh_node_morton_code_cuda* leaf_nodes_device, unsigned int leaf_node_num,
                                   int block_size);
void radix_sort(pt_bvh_node_morton_code_cuda* arrays, pt_bvh_node_morton_code_cuda* sorted_arrays, int number);

/* Whole-mesh Morton build on the current HIP device from host triangles (world space); same output
 * contract as pt_bvh_build (include/pt_host.h). Returns 0 on success. */
int pt_bvh_build_device(const pt_triangle* triangles, int n, int start_index, int leaf_size,
                        pt_bvh_node_device** nodes, int* node_num, int** leaf_indices, int* leaf_num);

#ifdef __cplusplus
}
#endif

#endif /* PT_BVH_H */
