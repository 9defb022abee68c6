/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see oracle_common.h).  C API of the CPU
 * restatement, loaded by tests/ and bench.py (cpu_baseline) through ctypes.
 */
#pragma once
#include <stdint.h>
#include "../include/hs_types.h"

#ifdef __cplusplus
extern "C" {
#endif
void hso_params_default(hs_params* p);
void* hso_ba_create(const hs_params* params, const hs_camera* cam, int nF, const hs_frame* frames,
                    const float* const* images, const hs_points* pts, const hs_residuals* rs, int nthreads);
void hso_ba_destroy(void* h);
int hso_ba_optimize(void* h, int iters, int allow_break, double* energies);
void hso_ba_iterate(void* h, int it0, int K, double* energies);
double hso_ba_linearize_all(void* h, int reset);
void hso_ba_apply_res(void* h);
void hso_ba_accumulate(void* h, int which, double* H, double* b);
void hso_ba_solve_system(void* h, int iteration, double* x_out);
void hso_ba_backup_state(void* h);
int hso_ba_do_step(void* h);
void hso_ba_get_residuals(void* h, uint8_t* state, uint8_t* new_state, double* energy, double* new_energy,
                          double* energy_with_outlier, float* resF, float* J_extra, float* JpJdF, float* center);
void hso_ba_get_points(void* h, float* idepth, float* step, float* HdiF, float* bdSumF, float* Hdd_accAF);
void hso_ba_get_frames(void* h, double* state, float* energyTH, double* pose7, double* calib_value4);
void hso_ba_get_precalc(void* h, float* out);
void hso_ba_get_nullspaces(void* h, double* N);
int hso_ba_res_in_A(void* h);
void hso_se3_exp(const double a[6], double out7[7]);
void hso_se3_log(const double in7[7], double a[6]);
void hso_se3_mul(const double a7[7], const double b7[7], double out7[7]);
void hso_se3_inverse(const double a7[7], double out7[7]);
void hso_se3_adj(const double a7[7], double A[36]);
void hso_se3_matrix(const double a7[7], double R9[9]);
#ifdef __cplusplus
}
#endif
