/* C ABI of the single-GPU engine: the device runtime API of the reference
 * (v4/comp.h:1-40: cudaInitGraph, cudaInitFrontiers, cudaExpandFrontier,
 * cudaCheckIntersect, cudaFreeGraph) with a handle instead of file-static
 * device pointers (v4/comp.cu:13-17) and device-resident state instead of
 * N-int host arrays copied every level (v4/comp.cu:94-106).
 * Every function returns 0 on success, -1 on error (bibfs_last_error()). */
#ifndef BIBFS_HIP_H
#define BIBFS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct bibfs_ctx bibfs_ctx;

typedef struct bibfs_result {
  int32_t found;
  int64_t hops;
  uint32_t meet;
  int32_t levels;
  uint64_t edges_inspected;
  double search_ms;
  double total_ms;
  size_t path_len; /* vertices written to the caller's path buffer */
} bibfs_result;

bibfs_ctx* bibfs_create(int device);
void bibfs_destroy(bibfs_ctx* ctx);
const char* bibfs_last_error(void);

/* cudaInitGraph parity: upload a host CSR (64-bit offsets) */
int bibfs_init_graph(bibfs_ctx* ctx, uint32_t n, uint64_t nnz, const uint64_t* row_off, const uint32_t* col);
/* upload an undirected edge list (u0 v0 u1 v1 ...) and build the CSR on the GPU */
int bibfs_init_graph_edges(bibfs_ctx* ctx, uint32_t n, uint64_t m, const uint32_t* uv);
/* load a .bin edge list file */
int bibfs_load_bin(bibfs_ctx* ctx, const char* path);

/* one-shot search; path may be NULL; path_cap in vertices */
int bibfs_search(bibfs_ctx* ctx, uint32_t src, uint32_t dst, bibfs_result* out, uint32_t* path, size_t path_cap);

/* step-wise interface (cudaInitFrontiers / cudaExpandFrontier / cudaCheckIntersect parity) */
int bibfs_init_frontiers(bibfs_ctx* ctx, uint32_t src, uint32_t dst);
int bibfs_expand_frontier(bibfs_ctx* ctx, int side, uint64_t* claimed, int* met);
int bibfs_check_intersect(bibfs_ctx* ctx, int* found);
int bibfs_finish(bibfs_ctx* ctx, bibfs_result* out, uint32_t* path, size_t path_cap);

/* cudaFreeGraph parity */
int bibfs_free_graph(bibfs_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* BIBFS_HIP_H */
