/* ORACLE — test infrastructure only (linked by tests/ through ctypes; never by
 * the product library).
 *
 * Plain-C restatement of the addressing the reference path performs on every
 * SAGEConv call (PyG 2.7.0 MessagePassing, flow='source_to_target', used at
 * /root/reference/src/models/blocks/sageblock.py:18): message e reads row
 * edge_index[0][e] and accumulates into row edge_index[1][e], edges visited in
 * their original order (CPU scatter_add_ order).  The product replaces that
 * per-call index_select/scatter addressing with a CSR built once per graph
 *; this file states what that CSR must be, bit for bit:
 *
 *   rowptr[i]..rowptr[i+1]   in-edges of node i (dst == i)
 *   col[k]                   their sources, in original edge order (stable)
 *   t_rowptr / t_col         the transpose: out-edges of node j (src == j),
 *                            their destinations, in original edge order
 *
 * A stable counting sort.  Node ids outside [0, N) are an error (PyG raises
 * on them), reported as -1 with no output written.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static void counting_sort(const int64_t* key, const int64_t* val, int64_t E,
                          int64_t N, int32_t* ptr, int32_t* out) {
    memset(ptr, 0, sizeof(int32_t) * (size_t)(N + 1));
    for (int64_t e = 0; e < E; ++e) ptr[key[e] + 1]++;
    for (int64_t i = 0; i < N; ++i) ptr[i + 1] += ptr[i];
    int32_t* cur = (int32_t*)malloc(sizeof(int32_t) * (size_t)(N > 0 ? N : 1));
    memcpy(cur, ptr, sizeof(int32_t) * (size_t)N);
    for (int64_t e = 0; e < E; ++e) out[cur[key[e]]++] = (int32_t)val[e];
    free(cur);
}

int csr_ref_build(const int64_t* edge_index, int64_t E, int64_t N,
                  int32_t* rowptr, int32_t* col, int32_t* t_rowptr, int32_t* t_col) {
    const int64_t* src = edge_index;
    const int64_t* dst = edge_index + E;
    for (int64_t e = 0; e < E; ++e)
        if (src[e] < 0 || src[e] >= N || dst[e] < 0 || dst[e] >= N) return -1;
    counting_sort(dst, src, E, N, rowptr, col);
    counting_sort(src, dst, E, N, t_rowptr, t_col);
    return 0;
}

/* fp32 mean aggregation in the reference's accumulation order (PyG
 * scatter(reduce='mean'): fp32 sums of messages in edge order, divided by the
 * fp32 in-degree clamped to 1).  x is [N, F] row-major fp32.  Used to pin the
 * GPU gather kernel bit for bit. */
void agg_ref_mean_f32(const float* x, int64_t N, int64_t F, const int32_t* rowptr,
                      const int32_t* col, float* out) {
    for (int64_t i = 0; i < N; ++i) {
        float* o = out + i * F;
        for (int64_t f = 0; f < F; ++f) o[f] = 0.0f;
        for (int32_t k = rowptr[i]; k < rowptr[i + 1]; ++k) {
            const float* xs = x + (int64_t)col[k] * F;
            for (int64_t f = 0; f < F; ++f) o[f] += xs[f];
        }
        float cnt = (float)(rowptr[i + 1] - rowptr[i]);
        if (cnt < 1.0f) cnt = 1.0f;
        for (int64_t f = 0; f < F; ++f) o[f] = o[f] / cnt;
    }
}
