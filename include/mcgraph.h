/*
 * mcgraph.h — C-ABI of the MI355X-native view-consensus graph path of
 * MaskClustering (libmcgraph.so, hand-written HIP kernels for gfx950).
 *
 * The library replaces the compute behind these reference interfaces
 * (paths relative to the reference repository):
 *
 *   graph/construction.py:7    mask_graph_construction      -> mc_scene_set_masks + mc_graph_build
 *   graph/construction.py:22   build_point_in_mask_matrix   -> mc_graph_build (S2)
 *   graph/construction.py:137  process_masks / :98 process_one_mask -> mc_graph_build (S3)
 *   graph/construction.py:80   get_observer_num_thresholds  -> mc_graph_build (S4) + mc_graph_get_thresholds
 *   graph/construction.py:66   init_nodes                   -> mc_graph_build (S5)
 *   graph/iterative_clustering.py:36 iterative_clustering   -> mc_cluster_run
 *   graph/iterative_clustering.py:13 update_graph           -> mc_cluster_run (pair counts + edge rule)
 *   graph/iterative_clustering.py:5  cluster_into_new_nodes -> mc_cluster_run (components)
 *   graph/node.py:24           Node.create_node_from_list   -> mc_cluster_run (on-device merge)
 *
 * Conventions
 *   - Every call returns 0 (MC_OK) or an MC_ERR_* code; mc_ctx_last_error()
 *     gives the message.  No call throws.
 *   - Host buffers are caller-owned; sizes are given by the *_get_info calls
 *     (two-call pattern: query sizes, then fill).
 *   - The context owns all device memory.  One context per device per host
 *     thread; no global state.  Work is enqueued on the context's HIP stream
 *     (its own, or the one given by mc_ctx_set_stream); getters synchronise it.
 *   - Masks are the reference's per-frame mask dicts flattened in frame
 *     order, ids in dict order (construction.py:46-60); frames whose mask
 *     union is empty are dropped like construction.py:50-51.
 */
#ifndef MCGRAPH_H
#define MCGRAPH_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MC_OK 0
#define MC_ERR_INVALID 1          /* bad argument / inconsistent input            */
#define MC_ERR_HIP 2              /* HIP runtime error                            */
#define MC_ERR_STATE 3            /* call out of order (e.g. cluster before build)*/
#define MC_ERR_EMPTY_OBSERVERS 4  /* np.percentile on empty (construction.py:89)   */
#define MC_ERR_UNSUPPORTED 5      /* size beyond a documented limit                */
#define MC_ERR_NO_NODES 6         /* torch.stack([]) (iterative_clustering.py:17)  */

typedef struct mc_ctx mc_ctx;

/* args fields read by graph/construction.py:119,125,132 */
typedef struct {
    double mask_visible_threshold;
    double contained_threshold;
    double undersegment_filter_threshold;
} mc_graph_params;

typedef struct {
    int64_t num_points;        /* P                                   */
    int32_t num_frames;        /* F (columns of the frame list)       */
    int32_t num_masks;         /* M: global masks (kept)              */
    int32_t num_undersegment;  /* |U|                                 */
    int32_t num_nodes0;        /* N0 = M - |U|                        */
    int64_t num_contained;     /* nnz of contained_masks after undo   */
    int64_t num_boundary;      /* |boundary_points|                   */
    int32_t num_thresholds;    /* len(observer_num_thresholds)        */
    int32_t threshold_status;  /* MC_OK or MC_ERR_EMPTY_OBSERVERS     */
} mc_graph_info;

typedef struct {
    int32_t num_iterations;    /* thresholds consumed                 */
    int32_t num_objects;       /* final nodes                         */
    int32_t num_nodes0;        /* nodes entering iteration 0          */
    int32_t reserved;
    int64_t num_object_points; /* sum over objects of |point_ids|     */
    int64_t num_object_contained; /* sum over objects of |contained|  */
    int64_t num_object_masks;  /* sum over objects of |mask_list|     */
} mc_cluster_info;

/* ---- context ------------------------------------------------------------ */
int mc_ctx_create(int device, mc_ctx **out);
void mc_ctx_destroy(mc_ctx *ctx);
int mc_ctx_set_stream(mc_ctx *ctx, void *hip_stream);   /* NULL = own stream */
void *mc_ctx_get_stream(mc_ctx *ctx);
int mc_ctx_synchronize(mc_ctx *ctx);
const char *mc_ctx_last_error(mc_ctx *ctx);
/* live per-kernel timing with HIP events on the context stream (bench/profiling) */
int mc_ctx_set_timing(mc_ctx *ctx, int enable);
int mc_ctx_set_timing_filter(mc_ctx *ctx, const char *kernel);  /* NULL/"" = every kernel group */
int mc_ctx_get_kernel_time(mc_ctx *ctx, const char *kernel, double *total_ms, int64_t *launches);
int mc_ctx_reset_kernel_times(mc_ctx *ctx);

/* ---- scene input (the S1 output: per-frame mask point sets) ---------------
 * mask_col/label/off are host arrays of length M_in, M_in, M_in+1.
 * mask_pts (length mask_off[M_in]) is a host pointer, or a device pointer
 * when pts_on_device != 0.  Point ids in [0, P); each mask's ids unique;
 * labels in [1, 65535] and unique within a frame; mask_col non-decreasing.  */
int mc_scene_set_masks(mc_ctx *ctx, int64_t num_points, int32_t num_frames, int32_t num_masks_in,
                       const int32_t *mask_col, const int32_t *mask_label, const int64_t *mask_off,
                       const int32_t *mask_pts, int pts_on_device);

/* ---- S2-S5: graph construction ------------------------------------------ */
int mc_graph_build(mc_ctx *ctx, const mc_graph_params *params);
int mc_graph_get_info(mc_ctx *ctx, mc_graph_info *info);
int mc_graph_get_global_masks(mc_ctx *ctx, int32_t *input_index /* M */);
int mc_graph_get_boundary(mc_ctx *ctx, uint8_t *flags /* P */);
int mc_graph_get_point_in_mask(mc_ctx *ctx, uint16_t *pim /* P*F, row-major */);
int mc_graph_get_point_frame_bits(mc_ctx *ctx, uint64_t *bits /* P*ceil(F/64) */);
int mc_graph_get_visible_frame_bits(mc_ctx *ctx, uint64_t *bits /* M*ceil(F/64) */);
int mc_graph_get_contained(mc_ctx *ctx, int64_t *row_off /* M+1 */, int32_t *col_idx /* nnz */);
int mc_graph_get_undersegment(mc_ctx *ctx, int32_t *ids /* |U| */);
int mc_graph_get_nodes0(mc_ctx *ctx, int32_t *mask_index /* N0 */);
int mc_graph_get_observer_hist(mc_ctx *ctx, uint64_t *hist /* F+1 */);
int mc_graph_get_thresholds(mc_ctx *ctx, float *thr /* 20 */, int32_t *is_int /* 20 */, int32_t *n);

/* get_observer_num_thresholds (construction.py:80-96) on an arbitrary
 * visible-frame matrix: rows of ceil(F/64) little-endian uint64 words.       */
int mc_observer_thresholds(mc_ctx *ctx, int32_t num_rows, int32_t num_frames, const uint64_t *vf_bits,
                           float *thr /* 20 */, int32_t *is_int /* 20 */, int32_t *n);

/* ---- S6 on arbitrary nodes (iterative_clustering on user Node lists) ------
 * Replaces the level-0 nodes: per node the visible-frame bits, the contained
 * mask ids (CSR, unique per row) and the point ids (CSR, unique per row).    */
int mc_nodes_set(mc_ctx *ctx, int32_t num_nodes, int32_t num_frames, int32_t num_masks,
                 int64_t num_points, const uint64_t *vf_bits, const int64_t *c_off,
                 const int32_t *c_idx, const int64_t *pt_off, const int32_t *pt_idx);

/* ---- S6: iterative view-consensus clustering ---------------------------
 * thresholds: host array of n values (np.float32 or the int 1), or NULL to
 * use the thresholds computed on the device by mc_graph_build (no host sync).
 * connect_threshold: args.view_consensus_threshold (compared in float32).   */
int mc_cluster_run(mc_ctx *ctx, const float *thresholds, int32_t n, double connect_threshold);
int mc_cluster_get_info(mc_ctx *ctx, mc_cluster_info *info);
int mc_cluster_get_level_sizes(mc_ctx *ctx, int32_t *sizes /* num_iterations+1 */);
int mc_cluster_get_partition(mc_ctx *ctx, int32_t iteration, int32_t *labels /* N_iteration */);
int mc_cluster_get_edge_counts(mc_ctx *ctx, int64_t *edges /* num_iterations */);
int mc_cluster_get_final_labels(mc_ctx *ctx, int32_t *labels /* N0: object of each level-0 node */);
int mc_cluster_get_objects(mc_ctx *ctx, uint64_t *vf_bits /* K*ceil(F/64) */,
                           int64_t *c_off /* K+1 */, int32_t *c_idx,
                           int64_t *pt_off /* K+1 */, int32_t *pt_idx,
                           int64_t *mask_off /* K+1 */, int32_t *mask_idx /* level-0 node ids */);

#ifdef __cplusplus
}
#endif
#endif /* MCGRAPH_H */
