/*
 * sldm_sage_cpu.h — C ABI of libsldm_sage_cpu.so: the SageBlock path for CPU
 * tensors, i.e. the reference's CPU mode (DEVICE = 'cpu',
 * /root/reference/main.py:58, test.py:18).  Host pointers, fp32 only,
 * OpenMP over rows.  Same algorithm and dropout hash as the gfx950 library
 * (include/sldm_sage.h); the layer GEMMs are the caller's (plain BLAS).
 * Each entry point replaces the same reference step as its GPU counterpart.
 */
#ifndef SLDM_SAGE_CPU_H
#define SLDM_SAGE_CPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

int sldm_cpu_abi_version(void);

/* sldm_csr_build on the host: ei = [2, E] int64 (row 0 sources); returns 1 on
 * an id outside [0, N) (outputs unspecified), else 0.  t_rowptr / t_col may
 * be NULL.  Replaces PyG propagate's addressing (sageblock.py:18). */
int sldm_cpu_csr_build(const int64_t* ei, int64_t E, int64_t N, int32_t* rowptr, int32_t* col,
                       int32_t* t_rowptr, int32_t* t_col);

/* sldm_gather_rows (fp32, CSR order): PyG index_select + scatter-mean
 * (A4-A5), or the transpose sum + addend of the backward (A8). */
void sldm_cpu_gather_rows(const float* x, int64_t ldx, const int32_t* rowptr, const int32_t* col,
                          int64_t nrows, int64_t feat, int mean, const float* addend,
                          int64_t lda, float* out, int64_t ldo);

/* d[i, :] /= max(1, deg_i) in place (the mean's backward). */
void sldm_cpu_scale_rows_by_inv_deg(float* d, int64_t ld, const int32_t* rowptr, int64_t nrows,
                                    int64_t feat);

/* sldm_post_fwd on the host: bias -> LayerNorm -> (Leaky)ReLU -> Dropout
 * (sageblock.py:11-13); out / xhat are [nrows, feat] contiguous. */
void sldm_cpu_post_fwd(const float* h, int64_t ldh, int64_t nrows, int64_t feat,
                       const float* bias, const float* gamma, const float* beta, float eps,
                       float slope, float drop_p, uint64_t seed, int64_t row_off, float* out,
                       float* xhat, float* rstd);

/* sldm_post_bwd on the host: dh and the dgamma / dbeta / dbias column sums. */
void sldm_cpu_post_bwd(const float* dout, const float* xhat, const float* rstd, int64_t nrows,
                       int64_t feat, const float* gamma, const float* beta, float slope,
                       float drop_p, uint64_t seed, int64_t row_off, float* dh, float* dgamma,
                       float* dbeta, float* dbias);

/* sldm_segment_pool on the host: PyG 2.7.0 global_mean_pool / global_max_pool
 * over the batch vector (grusage.py:3, :119-127, :185); batch [nrows] int64 in
 * [0, num_segments).  mean_out / max_out [B, feat] (either may be NULL), empty
 * segments give 0; max_divisor (fp32 [B, feat]) / max_first_row (int32
 * [B, feat]) as in include/sldm_sage.h (either may be NULL). */
void sldm_cpu_segment_pool(const float* x, int64_t ldx, const int64_t* batch, int64_t nrows,
                           int64_t num_segments, int64_t feat, float* mean_out, int64_t ld_mean,
                           float* max_out, int64_t ld_max, float* max_divisor,
                           int32_t* max_first_row);
void sldm_cpu_segment_pool_bwd(const float* x, int64_t ldx, const int64_t* batch, int64_t nrows,
                               int64_t num_segments, int64_t feat, const float* dmean,
                               int64_t ld_dmean, const float* max_out, int64_t ld_max,
                               const float* dmax, int64_t ld_dmax, const float* max_divisor,
                               const int32_t* max_first_row, float* dx, int64_t ld_dx);

#ifdef __cplusplus
}
#endif
#endif /* SLDM_SAGE_CPU_H */
