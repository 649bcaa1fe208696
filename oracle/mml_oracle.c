/*
 * oracle/mml_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker + timed CPU baseline).
 *
 * A plain-C restatement of MyMediaLite's matrix-factorization training path, written from
 * the reference's behaviour, never linked into the product.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * Parity status: the component arithmetic is pinned by the reference's own known-answer
 * tests (RowScalarProduct = 55, RowScalarProductWithRowDifference = 40, AUC cases, learn-rate
 * decay, DSGD partition shapes, StaticRatingData parse count; see tests/test_oracle.py).
 * The end-to-end trajectory (System.Random stream -> MathNet polar normals -> SGD) cannot be
 * run against the reference here (no CLR in the image); it is pinned only by
 * those component tests and the widely published System.Random(0) first draw.
 *
 * Build: oracle/Makefile (-O2 -ffp-contract=off: C# never contracts a*b+c into an FMA).
 */
#define _GNU_SOURCE
#include <math.h>
#include <stdatomic.h>
#include <stdint.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

/* ------------------------------------------------------------------------------------------
 * System.Random(int seed) -- .NET reference-source Knuth subtractive generator (BCL; called via
 * MyMediaLite.Random, src/MyMediaLite/Random.cs:23-64).  Restated from SURVEY.md A.2.
 * ---------------------------------------------------------------------------------------- */
typedef struct {
    int32_t seed_array[56];
    int32_t inext, inextp;
} ora_rng;

#define ORA_MBIG 2147483647
#define ORA_MSEED 161803398

void ora_rng_init(ora_rng* r, int32_t seed) {
    int32_t subtraction = (seed == INT32_MIN) ? INT32_MAX : (seed < 0 ? -seed : seed);
    int32_t mj = ORA_MSEED - subtraction;
    r->seed_array[55] = mj;
    int32_t mk = 1;
    for (int i = 1; i < 55; i++) {
        int ii = (21 * i) % 55;
        r->seed_array[ii] = mk;
        mk = mj - mk;
        if (mk < 0) mk += ORA_MBIG;
        mj = r->seed_array[ii];
    }
    for (int k = 1; k < 5; k++)
        for (int i = 1; i < 56; i++) {
            r->seed_array[i] -= r->seed_array[1 + (i + 30) % 55];
            if (r->seed_array[i] < 0) r->seed_array[i] += ORA_MBIG;
        }
    r->inext = 0;
    r->inextp = 21;
}

size_t ora_rng_sizeof(void) { return sizeof(ora_rng); }

int32_t ora_rng_internal_sample(ora_rng* r) {
    int32_t a = r->inext + 1, b = r->inextp + 1;
    if (a >= 56) a = 1;
    if (b >= 56) b = 1;
    int32_t v = r->seed_array[a] - r->seed_array[b];
    if (v == ORA_MBIG) v--;
    if (v < 0) v += ORA_MBIG;
    r->seed_array[a] = v;
    r->inext = a;
    r->inextp = b;
    return v;
}

double ora_rng_next_double(ora_rng* r) { return ora_rng_internal_sample(r) * (1.0 / ORA_MBIG); }

/* Random.Next(maxValue) = (int)(Sample() * maxValue) */
int32_t ora_rng_next(ora_rng* r, int32_t max_value) {
    return (int32_t)(ora_rng_next_double(r) * max_value);
}

/* MathNet.Numerics 3.15 Normal.Sample(): polar transform, second variate discarded. */
double ora_normal(ora_rng* r, double mean, double stddev) {
    for (;;) {
        double a = ora_rng_next_double(r);
        double b = ora_rng_next_double(r);
        double v1 = 2.0 * a - 1.0;
        double v2 = 2.0 * b - 1.0;
        double rr = v1 * v1 + v2 * v2;
        if (rr >= 1.0 || rr == 0.0) continue;
        double fac = sqrt(-2.0 * log(rr) / rr);
        return mean + stddev * (v1 * fac);
    }
}

/* MatrixExtensions.InitNormal (DataType/MatrixExtensions.cs:62-69): row-major fill, cast to float */
void ora_fill_normal(ora_rng* r, float* out, int64_t n, double mean, double stddev) {
    for (int64_t i = 0; i < n; i++) out[i] = (float)ora_normal(r, mean, stddev);
}

/* Utils.Shuffle (src/MyMediaLite/Utils.cs:52-64): i = n-1 .. 0, r = Next(i+1), swap */
void ora_shuffle_i32(ora_rng* r, int32_t* a, int64_t n) {
    for (int64_t i = n - 1; i >= 0; i--) {
        int32_t j = ora_rng_next(r, (int32_t)(i + 1));
        int32_t t = a[i];
        a[i] = a[j];
        a[j] = t;
    }
}

/* ------------------------------------------------------------------------------------------
 * DataType/MatrixExtensions.cs row kernels (known answers: tests/test_oracle.py)
 * ---------------------------------------------------------------------------------------- */
/* RowScalarProduct(Matrix<float>,int,Matrix<float>,int), MatrixExtensions.cs:224-241: float acc */
float ora_row_scalar_product(const float* m1, int i, const float* m2, int j, int k) {
    float result = 0.0f;
    const float* a = m1 + (int64_t)i * k;
    const float* b = m2 + (int64_t)j * k;
    for (int c = 0; c < k; c++) result += a[c] * b[c];
    return result;
}

/* RowScalarProductWithRowDifference, MatrixExtensions.cs:276-298: float products, double acc */
double ora_row_scalar_product_with_row_difference(const float* m1, int i, const float* m2, int j,
                                                  const float* m3, int l, int k) {
    double result = 0.0;
    const float* a = m1 + (int64_t)i * k;
    const float* b = m2 + (int64_t)j * k;
    const float* c3 = m3 + (int64_t)l * k;
    for (int c = 0; c < k; c++) result += (double)(a[c] * (b[c] - c3[c]));
    return result;
}

/* ------------------------------------------------------------------------------------------
 * BiasedMatrixFactorization (RatingPrediction/BiasedMatrixFactorization.cs)
 * ---------------------------------------------------------------------------------------- */
enum { ORA_LOSS_RMSE = 0, ORA_LOSS_MAE = 1, ORA_LOSS_LOGISTIC = 2 };

typedef struct {
    int32_t k;
    int32_t loss;
    int32_t frequency_regularization;
    int32_t update_user;
    int32_t update_item;
    float global_bias;
    float min_rating;
    float rating_range_size;
    float learn_rate;      /* current_learnrate */
    float bias_learn_rate; /* BiasLearnRate */
    float bias_reg;        /* BiasReg */
    float reg_u;           /* RegU */
    float reg_i;           /* RegI */
} ora_bmf_params;

size_t ora_bmf_params_sizeof(void) { return sizeof(ora_bmf_params); }

/* BiasedMatrixFactorization.Iterate(IList<int>,bool,bool), :264-310 (with SetupLoss :247-261) */
void ora_bmf_iterate(const ora_bmf_params* p, const int32_t* users, const int32_t* items,
                     const float* values, const int32_t* idx, int64_t n_idx, float* U, float* V,
                     float* bu, float* bi, const int32_t* count_by_user,
                     const int32_t* count_by_item) {
    const int k = p->k;
    const float lr = p->learn_rate;
    enum { AHEAD = 32 };  /* rows requested AHEAD ratings early: a cache hint, the order is kept */
    for (int64_t n = 0; n < n_idx; n++) {
        if (n + AHEAD < n_idx) {
            const int32_t ahead = idx[n + AHEAD];
            const char* pu = (const char*)(U + (int64_t)users[ahead] * k);
            const char* pv = (const char*)(V + (int64_t)items[ahead] * k);
            for (int c = 0; c < k * 4; c += 64) {
                __builtin_prefetch(pu + c, 1);
                __builtin_prefetch(pv + c, 1);
            }
            __builtin_prefetch(bu + users[ahead], 1);
            __builtin_prefetch(bi + items[ahead], 1);
        }
        int32_t index = idx[n];
        int32_t u = users[index];
        int32_t i = items[index];
        float* Uu = U + (int64_t)u * k;
        float* Vi = V + (int64_t)i * k;

        float dot = 0.0f;
        for (int c = 0; c < k; c++) dot += Uu[c] * Vi[c];
        float score_f = ((p->global_bias + bu[u]) + bi[i]) + dot;
        double score = (double)score_f;
        double sig = 1.0 / (1.0 + exp(-score));
        double prediction = (double)p->min_rating + sig * (double)p->rating_range_size;
        double err = (double)values[index] - prediction;

        float g;
        if (p->loss == ORA_LOSS_MAE) {
            double sgn = (err > 0) ? 1.0 : ((err < 0) ? -1.0 : 0.0);
            g = (float)(sgn * sig * (1.0 - sig) * (double)p->rating_range_size);
        } else if (p->loss == ORA_LOSS_LOGISTIC) {
            g = (float)err;
        } else {
            g = (float)(err * sig * (1.0 - sig) * (double)p->rating_range_size);
        }

        float reg_u = p->reg_u, reg_i = p->reg_i;
        if (p->frequency_regularization) {
            reg_u = (float)((double)p->reg_u / sqrt((double)count_by_user[u]));
            reg_i = (float)((double)p->reg_i / sqrt((double)count_by_item[i]));
        }

        const float blr = p->bias_learn_rate * lr;
        if (p->update_user) bu[u] += blr * (g - (p->bias_reg * reg_u) * bu[u]);
        if (p->update_item) bi[i] += blr * (g - (p->bias_reg * reg_i) * bi[i]);

        for (int f = 0; f < k; f++) {
            double u_f = (double)Uu[f];
            double i_f = (double)Vi[f];
            if (p->update_user) {
                double delta_u = (double)g * i_f - (double)reg_u * u_f;
                Uu[f] += (float)((double)lr * delta_u);
            }
            if (p->update_item) {
                double delta_i = (double)g * u_f - (double)reg_i * i_f;
                Vi[f] += (float)((double)lr * delta_i);
            }
        }
    }
}

/* Hogwild's staleness, restated for the Hogwild bands of the tests (not a reference behaviour):
 * the stream idx[0 .. n_idx) is cut into W contiguous chunks, one per stream (a wavefront of the
 * GPU kernel); at step t every stream takes its next R ratings.  All ratings of a step read the
 * model as it was before the step (ora_bmf_iterate's arithmetic on those values), then their
 * results are written in stream order, so a later stream's write of a row replaces an earlier
 * one's (the lost update of two wavefronts writing one row).  W = 1, R = 1 is ora_bmf_iterate.
 * threads: how many threads compute a step's updates (the result does not depend on it). */
void ora_bmf_iterate_lockstep(const ora_bmf_params* p, const int32_t* users, const int32_t* items,
                              const float* values, const int32_t* idx, int64_t n_idx, float* U,
                              float* V, float* bu, float* bi, const int32_t* count_by_user,
                              const int32_t* count_by_item, int32_t W, int32_t R,
                              int32_t threads) {
    const int k = p->k;
    const int nt = threads > 0 ? threads : 1;
    const int64_t per = (n_idx + W - 1) / W;
    const int64_t cap = (int64_t)W * R;
    float* nu = (float*)malloc(sizeof(float) * (size_t)cap * (k + 1));
    float* nv = (float*)malloc(sizeof(float) * (size_t)cap * (k + 1));
    int32_t* su = (int32_t*)malloc(sizeof(int32_t) * (size_t)cap);
    int32_t* si = (int32_t*)malloc(sizeof(int32_t) * (size_t)cap);
    int64_t* sp = (int64_t*)malloc(sizeof(int64_t) * (size_t)cap);
    for (int64_t t = 0; t * R < per; ++t) {
        int64_t m = 0;  /* the step's ratings in stream order */
        for (int32_t w = 0; w < W; ++w)
            for (int32_t r = 0; r < R; ++r) {
                const int64_t pos = (int64_t)w * per + t * R + r;
                if (t * R + r >= per || pos >= n_idx) continue;
                sp[m++] = pos;
            }
        /* every rating of the step from the model before the step: independent, so on threads
         * (OpenMP, `threads` of them); the results land in the step's buffers, the model is not
         * touched */
#pragma omp parallel for schedule(static) num_threads(nt) if (nt > 1)
        for (int64_t x = 0; x < m; ++x) {
            const int32_t index = idx[sp[x]], u = users[index], i = items[index];
            float* Uo = nu + x * (k + 1);
            float* Vo = nv + x * (k + 1);
            memcpy(Uo, U + (int64_t)u * k, sizeof(float) * k);
            memcpy(Vo, V + (int64_t)i * k, sizeof(float) * k);
            float bu1 = bu[u], bi1 = bi[i];
            const int32_t zero = 0;  // the rating's rows, copied: row 0 of Uo / Vo
            ora_bmf_iterate(p, &zero, &zero, values + index, &zero, 1, Uo, Vo, &bu1, &bi1,
                            count_by_user ? count_by_user + u : NULL,
                            count_by_item ? count_by_item + i : NULL);
            Uo[k] = bu1;
            Vo[k] = bi1;
            su[x] = u;
            si[x] = i;
        }
        for (int64_t x = 0; x < m; ++x) {  /* writes in stream order: the last one stays */
            if (p->update_user) {
                memcpy(U + (int64_t)su[x] * k, nu + x * (k + 1), sizeof(float) * k);
                bu[su[x]] = nu[x * (k + 1) + k];
            }
            if (p->update_item) {
                memcpy(V + (int64_t)si[x] * k, nv + x * (k + 1), sizeof(float) * k);
                bi[si[x]] = nv[x * (k + 1) + k];
            }
        }
    }
    free(nu);
    free(nv);
    free(su);
    free(si);
    free(sp);
}

/* y summed over the user's rated items (MatrixExtensions.SumOfRows, DataType/MatrixExtensions.cs:
 * 125-135: float accumulation in list order), / sqrt(count) in double, cast to float -- the user
 * vector of SigmoidItemAsymmetricFactorModel (Iterate :104-107, PrecomputeUserFactors :316-331) */
static void ora_iafm_user_vector(const float* Y, int k, const int64_t* rated_off,
                                 const int32_t* rated_items, int32_t u, float* vec, double* norm) {
    const int64_t b = rated_off[u], e = rated_off[u + 1];
    for (int f = 0; f < k; f++) vec[f] = 0.0f;
    for (int64_t t = b; t < e; t++) {
        const float* row = Y + (int64_t)rated_items[t] * k;
        for (int f = 0; f < k; f++) vec[f] += row[f];
    }
    *norm = sqrt((double)(e - b));
    for (int f = 0; f < k; f++) vec[f] = (float)((double)vec[f] / *norm);
}

/* The asymmetric models' Iterate(IList<int>,bool,bool).  Slot 0: per user the items rated
 * (ITransductiveRatingPredictor.ItemsRatedByUser, :63-79: training items in rating-index order,
 * then AdditionalFeedback's, distinct) over Y = y [n_items x k] with y_reg; slot 1: per item the
 * users who rated it (UsersWhoRated, :40-55) over X = x [n_users x k] with x_reg.
 *   mode 0 SigmoidItemAsymmetricFactorModel (SigmoidItemAsymmetricFactorModel.cs:91-147):
 *          user vector from y; trains V_i (RowScalarProduct, float) and y
 *   mode 1 SigmoidUserAsymmetricFactorModel (SigmoidUserAsymmetricFactorModel.cs:91-144):
 *          item vector from x; trains U_u and x
 *   mode 2 SigmoidCombinedAsymmetricFactorModel (SigmoidCombinedAsymmetricFactorModel.cs:
 *          108-182): both vectors; VectorExtensions.ScalarProduct (double sum, VectorExtensions.cs:
 *          30-38); trains x (from the user vector) and y (from the item vector)
 *   mode 3 SVDPlusPlus (SVDPlusPlus.cs:157-212): user vector = (float)(y sum / norm + p_u); no
 *          sigmoid: err = r - prediction drives the (float)err bias steps and the double p_u,
 *          V_i and y steps
 *   mode 4 SigmoidSVDPlusPlus (SigmoidSVDPlusPlus.cs:111-173): the same vector with the sigmoid
 *          link and gradient_common (float update expressions)
 * P: p [n_users x k] (modes 3, 4).  vu, vi: k floats of scratch each. */
void ora_asym_iterate(const ora_bmf_params* p, const int32_t* users, const int32_t* items,
                      const float* values, const int32_t* idx, int64_t n_idx, float* U, float* V,
                      float* bu, float* bi, const int32_t* count_by_user,
                      const int32_t* count_by_item, float* Y, const int64_t* off_u,
                      const int32_t* ids_u, const float* y_reg, float* X, const int64_t* off_i,
                      const int32_t* ids_i, const float* x_reg, float* vu, float* vi,
                      int32_t mode, float* P) {
    const int k = p->k;
    const float lr = p->learn_rate;
    for (int64_t n = 0; n < n_idx; n++) {
        const int32_t index = idx[n];
        const int32_t u = users[index], i = items[index];
        double norm_u = 1.0, norm_i = 1.0;
        if (mode >= 3) { /* p_plus_y_sum_vector (SVDPlusPlus.cs:166-170) */
            const int64_t b = off_u[u], e = off_u[u + 1];
            for (int f = 0; f < k; f++) vu[f] = 0.0f;
            for (int64_t t = b; t < e; t++)
                for (int f = 0; f < k; f++) vu[f] += Y[(int64_t)ids_u[t] * k + f];
            norm_u = sqrt((double)(e - b));
            for (int f = 0; f < k; f++)
                vu[f] = (float)((double)vu[f] / norm_u + (double)P[(int64_t)u * k + f]);
        } else if (mode != 1) {
            ora_iafm_user_vector(Y, k, off_u, ids_u, u, vu, &norm_u);
        }
        if (mode == 1 || mode == 2) ora_iafm_user_vector(X, k, off_i, ids_i, i, vi, &norm_i);
        float* Ui = U + (int64_t)u * k;
        float* Vi = V + (int64_t)i * k;
        double score = (double)((p->global_bias + bu[u]) + bi[i]); /* float sum */
        if (mode == 0 || mode >= 3) { /* item_factors.RowScalarProduct(i, vector) */
            float dot = 0.0f;
            for (int f = 0; f < k; f++) dot += Vi[f] * vu[f];
            score += (double)dot;
        } else if (mode == 1) { /* user_factors.RowScalarProduct(u, x_sum) */
            float dot = 0.0f;
            for (int f = 0; f < k; f++) dot += Ui[f] * vi[f];
            score += (double)dot;
        } else {                /* ScalarProduct(y_sum, x_sum) */
            double dot = 0.0;
            for (int f = 0; f < k; f++) dot += (double)(vu[f] * vi[f]);
            score += (double)(float)dot;
        }
        double sig = 0.0, err;
        float g;
        if (mode == 3) {
            err = (double)values[index] - score;
        } else {
            sig = 1.0 / (1.0 + exp(-score));
            err = (double)values[index] -
                  ((double)p->min_rating + sig * (double)p->rating_range_size);
        }
        if (mode == 3) {
            g = (float)err;
        } else if (p->loss == ORA_LOSS_MAE) {
            double sgn = (err > 0) ? 1.0 : ((err < 0) ? -1.0 : 0.0);
            g = (float)(sgn * sig * (1.0 - sig) * (double)p->rating_range_size);
        } else if (p->loss == ORA_LOSS_LOGISTIC) {
            g = (float)err;
        } else {
            g = (float)(err * sig * (1.0 - sig) * (double)p->rating_range_size);
        }
        float reg_u = p->reg_u, reg_i = p->reg_i;
        if (p->frequency_regularization) {
            reg_u = (float)((double)p->reg_u / sqrt((double)count_by_user[u]));
            reg_i = (float)((double)p->reg_i / sqrt((double)count_by_item[i]));
        }
        const float blr = p->bias_learn_rate * lr;
        if (p->update_user) bu[u] += blr * (g - (p->bias_reg * reg_u) * bu[u]);
        if (p->update_item) bi[i] += blr * (g - (p->bias_reg * reg_i) * bi[i]);
        const double ngc_u = (double)g / norm_u, ngc_i = (double)g / norm_i;
        for (int f = 0; f < k; f++) {
            if (mode >= 3) {
                const float i_f = Vi[f];
                float* pf = P + (int64_t)u * k + f;
                if (p->update_user) {
                    const double delta_u = mode == 3 ? err * (double)i_f - (double)(reg_u * *pf)
                                                     : (double)(g * i_f - reg_u * *pf);
                    *pf += (float)((double)lr * delta_u);
                }
                if (p->update_item) {
                    const double delta_i = mode == 3 ? err * (double)vu[f] - (double)(reg_i * i_f)
                                                     : (double)(g * vu[f] - reg_i * i_f);
                    Vi[f] += (float)((double)lr * delta_i);
                    const double common = (mode == 3 ? err / norm_u : ngc_u) * (double)i_f;
                    for (int64_t t = off_u[u]; t < off_u[u + 1]; t++) {
                        float* yj = Y + (int64_t)ids_u[t] * k + f;
                        *yj += (float)((double)lr * (common - (double)(y_reg[ids_u[t]] * *yj)));
                    }
                }
            } else if (mode == 0) {
                const float i_f = Vi[f];
                if (!p->update_item) continue;
                const double delta_i = (double)(g * vu[f] - reg_i * i_f); /* float expression */
                Vi[f] += (float)((double)lr * delta_i);
                const double common = ngc_u * (double)i_f;
                for (int64_t t = off_u[u]; t < off_u[u + 1]; t++) {
                    float* yj = Y + (int64_t)ids_u[t] * k + f;
                    *yj += (float)((double)lr * (common - (double)(y_reg[ids_u[t]] * *yj)));
                }
            } else if (mode == 1) {
                const float u_f = Ui[f];
                if (!p->update_user) continue;
                const double delta_u = (double)(g * vi[f] - reg_u * u_f);
                Ui[f] += (float)((double)lr * delta_u);
                const double common = ngc_i * (double)u_f;
                for (int64_t t = off_i[i]; t < off_i[i + 1]; t++) {
                    float* xo = X + (int64_t)ids_i[t] * k + f;
                    *xo += (float)((double)lr * (common - (double)(x_reg[ids_i[t]] * *xo)));
                }
            } else {
                const float u_f = vu[f], i_f = vi[f];
                if (p->update_user) {
                    const double common = ngc_i * (double)u_f;
                    for (int64_t t = off_i[i]; t < off_i[i + 1]; t++) {
                        float* xo = X + (int64_t)ids_i[t] * k + f;
                        *xo += (float)((double)lr * (common - (double)(x_reg[ids_i[t]] * *xo)));
                    }
                }
                if (p->update_item) {
                    const double common = ngc_u * (double)i_f;
                    for (int64_t t = off_u[u]; t < off_u[u + 1]; t++) {
                        float* yj = Y + (int64_t)ids_u[t] * k + f;
                        *yj += (float)((double)lr * (common - (double)(y_reg[ids_u[t]] * *yj)));
                    }
                }
            }
        }
    }
}

/* PrecomputeUserFactors (:305-331): U[u] = the user vector; users without items keep zeros.
 * P != NULL: SVDPlusPlus.PrecomputeFactors (SVDPlusPlus.cs:230-246), (float)(sum / norm + p) */
void ora_iafm_user_factors(const float* Y, int k, int32_t n_users, const int64_t* rated_off,
                           const int32_t* rated_items, float* U, const float* P) {
    for (int32_t u = 0; u < n_users; u++) {
        double norm;
        float* row = U + (int64_t)u * k;
        const int64_t b = rated_off[u], e = rated_off[u + 1];
        if (e == b) {
            for (int f = 0; f < k; f++) row[f] = 0.0f;
            continue;
        }
        if (!P) {
            ora_iafm_user_vector(Y, k, rated_off, rated_items, u, row, &norm);
            continue;
        }
        for (int f = 0; f < k; f++) row[f] = 0.0f;
        for (int64_t t = b; t < e; t++)
            for (int f = 0; f < k; f++) row[f] += Y[(int64_t)rated_items[t] * k + f];
        norm = sqrt((double)(e - b));
        for (int f = 0; f < k; f++)
            row[f] = (float)((double)row[f] / norm + (double)P[(int64_t)u * k + f]);
    }
}

/* BiasedMatrixFactorization.Predict(int,int), :313-325 (score accumulated in double) */
float ora_bmf_predict1(int32_t u, int32_t i, int32_t n_users, int32_t n_items, int k,
                       const float* U, const float* V, const float* bu, const float* bi,
                       float global_bias, float min_rating, float range) {
    double score = (double)global_bias;
    if (u < n_users) score += (double)bu[u];
    if (i < n_items) score += (double)bi[i];
    if (u < n_users && i < n_items) score += (double)ora_row_scalar_product(U, u, V, i, k);
    return (float)((double)min_rating + (1.0 / (1.0 + exp(-score))) * (double)range);
}

void ora_bmf_predict(const int32_t* users, const int32_t* items, int64_t n, int32_t n_users,
                     int32_t n_items, int k, const float* U, const float* V, const float* bu,
                     const float* bi, float global_bias, float min_rating, float range,
                     float* out) {
    for (int64_t x = 0; x < n; x++)
        out[x] = ora_bmf_predict1(users[x], items[x], n_users, n_items, k, U, V, bu, bi,
                                  global_bias, min_rating, range);
}

/* Eval/Ratings.cs:96-139: float error, float square, double sum; RMSE/MAE cast to float.
 * out[0] = RMSE, out[1] = MAE */
void ora_rating_eval(const float* predictions, const float* values, int64_t n, float* out) {
    double rmse = 0.0, mae = 0.0;
    for (int64_t x = 0; x < n; x++) {
        float error = predictions[x] - values[x];
        rmse += (double)(error * error);
        mae += (double)fabsf(error);
    }
    out[0] = (float)sqrt(rmse / (double)n);
    out[1] = (float)(mae / (double)n);
}

/* BiasedMatrixFactorization.ComputeLoss + ComputeObjective (:496-552), RMSE.ComputeSquaredErrorSum
 * (Eval/Measures/RMSE.cs:32-38), MAE.ComputeAbsoluteErrorSum (MAE.cs:32-38), LogisticLoss.ComputeSum
 * (LogisticLoss.cs:34-55).  out[0] = loss, out[1] = complexity (both double, unrounded). */
void ora_bmf_objective(const int32_t* users, const int32_t* items, const float* values, int64_t n,
                       int32_t n_users, int32_t n_items, int k, const float* U, const float* V,
                       const float* bu, const float* bi, float global_bias, float min_rating,
                       float range, int loss_kind, float reg_u, float reg_i, float bias_reg,
                       int frequency_regularization, const int32_t* cnt_u, const int32_t* cnt_i,
                       double* out) {
    double loss = 0.0;
    for (int64_t x = 0; x < n; x++) {
        float p = ora_bmf_predict1(users[x], items[x], n_users, n_items, k, U, V, bu, bi,
                                   global_bias, min_rating, range);
        if (loss_kind == 0) {
            double d = (double)(p - values[x]);
            loss += pow(d, 2.0);
        } else if (loss_kind == 1) {
            loss += fabs((double)(p - values[x]));
        } else {
            double prediction = ((double)p - (double)min_rating) / (double)range;
            if (prediction < 0.0) prediction = 0.0;
            if (prediction > 1.0) prediction = 1.0;
            double actual = (double)((values[x] - min_rating) / range);
            loss -= actual * log(prediction);
            loss -= (1 - actual) * log(1 - prediction);
        }
    }
    double complexity = 0.0;
    for (int side = 0; side < 2; side++) {
        int32_t rows = side == 0 ? n_users : n_items;
        const float* M = side == 0 ? U : V;
        const float* b = side == 0 ? bu : bi;
        const int32_t* cnt = side == 0 ? cnt_u : cnt_i;
        float reg = side == 0 ? reg_u : reg_i;
        for (int32_t r = 0; r < rows; r++) {
            double sq = 0.0;
            for (int f = 0; f < k; f++) sq += pow((double)M[(int64_t)r * k + f], 2.0);
            double norm2 = pow(sqrt(sq), 2.0);  /* Math.Pow(EuclideanNorm(row), 2) */
            if (frequency_regularization) {
                if (cnt[r] > 0) {
                    double w = (double)reg / sqrt((double)cnt[r]);
                    complexity += w * norm2;
                    complexity += w * (double)bias_reg * pow((double)b[r], 2.0);
                }
            } else {
                float w = (float)cnt[r] * reg;           /* int * float -> float in C# */
                float wb = (float)cnt[r] * reg * bias_reg;
                complexity += (double)w * norm2;
                complexity += (double)wb * pow((double)b[r], 2.0);
            }
        }
    }
    out[0] = loss;
    out[1] = complexity;
}

/* BiasedMatrixFactorization.FoldIn (:447-492) for one user, its rated_items already shuffled and
 * `factors` already drawn (InitNormal, then Shuffle, on the host RNG).  Uses LearnRate (not the
 * decayed current rate), no decay; the bias step and the factor delta are float expressions (float
 * operands), widened to double for the factor step.  out[0] = user bias, out[1..k] = factors. */
void ora_bmf_fold_in(const ora_bmf_params* p, int64_t n, const int32_t* items, const float* values,
                     int32_t num_iter, const float* V, const float* bi, const float* init_factors,
                     float* out) {
    const int k = p->k;
    float* factors = out + 1;
    for (int f = 0; f < k; f++) factors[f] = init_factors[f];
    float user_bias = 0.0f;
    const float reg_weight = p->frequency_regularization
                                 ? (float)((double)p->reg_u / sqrt((double)n))
                                 : p->reg_u;
    for (int32_t it = 0; it < num_iter; it++)
        for (int64_t x = 0; x < n; x++) {
            const int32_t item = items[x];
            const float* Vi = V + (int64_t)item * k;
            float dot = 0.0f;
            for (int f = 0; f < k; f++) dot += Vi[f] * factors[f];
            const double score = (double)(((p->global_bias + user_bias) + bi[item]) + dot);
            const double sig = 1.0 / (1.0 + exp(-score));
            const double prediction = (double)p->min_rating + sig * (double)p->rating_range_size;
            const double err = (double)values[x] - prediction;
            float g;
            if (p->loss == ORA_LOSS_MAE) {
                const double sgn = (err > 0) ? 1.0 : ((err < 0) ? -1.0 : 0.0);
                g = (float)(sgn * sig * (1.0 - sig) * (double)p->rating_range_size);
            } else if (p->loss == ORA_LOSS_LOGISTIC) {
                g = (float)err;
            } else {
                g = (float)(err * sig * (1.0 - sig) * (double)p->rating_range_size);
            }
            user_bias += p->bias_learn_rate * p->learn_rate *
                         (g - p->bias_reg * reg_weight * user_bias);
            for (int f = 0; f < k; f++) {
                const float u_f = factors[f];
                const float i_f = Vi[f];
                const double delta_u = (double)(g * i_f - reg_weight * u_f);
                factors[f] += (float)((double)p->learn_rate * delta_u);
            }
        }
    out[0] = user_bias;
}

/* BiasedMatrixFactorization.Predict(float[] user_vector, int item_id) (:327-335) */
float ora_bmf_predict_vector(const ora_bmf_params* p, const float* user_vector, int32_t item,
                             int32_t n_items, const float* V, const float* bi) {
    double score = (double)(p->global_bias + user_vector[0]);
    if (item < n_items) {
        float dot = 0.0f;
        for (int f = 0; f < p->k; f++) dot += V[(int64_t)item * p->k + f] * user_vector[1 + f];
        score += (double)(bi[item] + dot);
    }
    return (float)((double)p->min_rating +
                   1.0 / (1.0 + exp(-score)) * (double)p->rating_range_size);
}

/* ----------------------------------------------------------------------------------------
 * MatrixFactorization (RatingPrediction/MatrixFactorization.cs): the plain model, no biases
 * ---------------------------------------------------------------------------------------- */

/* MatrixFactorization.Iterate(IList<int>,bool,bool), :166-196, with Predict(u, i, false) :205-217:
 * err = r - (global_bias + RowScalarProduct) in float; delta = err * i_f - Regularization * u_f
 * evaluated in float (all operands are float in C#) and widened to double; Inc adds
 * (float)(current_learnrate * delta).  u_f and i_f are read before either row is written. */
void ora_mf_iterate(int k, float global_bias, float learn_rate, float regularization,
                    int update_user, int update_item, const int32_t* users, const int32_t* items,
                    const float* values, const int32_t* idx, int64_t n_idx, float* U, float* V) {
    for (int64_t n = 0; n < n_idx; n++) {
        const int32_t index = idx[n];
        float* Uu = U + (int64_t)users[index] * k;
        float* Vi = V + (int64_t)items[index] * k;
        float dot = 0.0f;
        for (int c = 0; c < k; c++) dot += Uu[c] * Vi[c];
        const float err = values[index] - (global_bias + dot);
        for (int f = 0; f < k; f++) {
            const float u_f = Uu[f];
            const float i_f = Vi[f];
            if (update_user) {
                const double delta_u = (double)(err * i_f - regularization * u_f);
                Uu[f] += (float)((double)learn_rate * delta_u);
            }
            if (update_item) {
                const double delta_i = (double)(err * u_f - regularization * i_f);
                Vi[f] += (float)((double)learn_rate * delta_i);
            }
        }
    }
}

/* MatrixFactorization.FoldIn (:326-351) for one user (rated_items shuffled, user_vector drawn by
 * the host): double lr = LearnRate, multiplied by Decay after every pass; err and delta in float. */
void ora_mf_fold_in(int k, float global_bias, float learn_rate, float decay, float regularization,
                    int64_t n, const int32_t* items, const float* values, int32_t num_iter,
                    const float* V, const float* init_factors, float* out) {
    for (int f = 0; f < k; f++) out[f] = init_factors[f];
    double lr = (double)learn_rate;
    for (int32_t it = 0; it < num_iter; it++) {
        for (int64_t x = 0; x < n; x++) {
            const float* Vi = V + (int64_t)items[x] * k;
            float dot = 0.0f;
            for (int f = 0; f < k; f++) dot += Vi[f] * out[f];
            const float err = values[x] - (global_bias + dot);
            for (int f = 0; f < k; f++) {
                const float u_f = out[f];
                const float i_f = Vi[f];
                const double delta_u = (double)(err * i_f - regularization * u_f);
                out[f] += (float)(lr * delta_u);
            }
        }
        lr *= (double)decay;
    }
}

/* MatrixFactorization.Predict(float[] user_vector, int item_id) (:222-241), bound */
float ora_mf_predict_vector(int k, float global_bias, float min_rating, float max_rating,
                           const float* user_vector, int32_t item, const float* V) {
    float dot = 0.0f;
    for (int f = 0; f < k; f++) dot += V[(int64_t)item * k + f] * user_vector[f];
    float r = global_bias + dot;
    if (r > max_rating) r = max_rating;
    if (r < min_rating) r = min_rating;
    return r;
}

/* MatrixFactorization.Predict(int,int), :251-258 (+ Predict(u, i, true) :205-217): global_bias for
 * ids beyond the model, else global_bias + RowScalarProduct clipped to [MinRating, MaxRating]. */
void ora_mf_predict(const int32_t* users, const int32_t* items, int64_t n, int32_t n_users,
                    int32_t n_items, int k, const float* U, const float* V, float global_bias,
                    float min_rating, float max_rating, float* out) {
    for (int64_t x = 0; x < n; x++) {
        const int32_t u = users[x], i = items[x];
        if (u >= n_users || i >= n_items) {
            out[x] = global_bias;
            continue;
        }
        float r = global_bias + ora_row_scalar_product(U, u, V, i, k);
        if (r > max_rating) r = max_rating;
        if (r < min_rating) r = min_rating;
        out[x] = r;
    }
}

/* ----------------------------------------------------------------------------------------
 * SocialMF (RatingPrediction/SocialMF.cs): BiasedMatrixFactorization with a social-network
 * regulariser, trained by full-batch gradient descent (Iterate(IList...) -> IterateBatch :77-194).
 * user_connections rows (HashSet enumeration = insertion order) as conn CSR over n_conn rows;
 * rev = its Transpose() (SparseBooleanMatrix.cs:200-207: rows filled by ascending source row).
 * p->learn_rate = LearnRate (IterateBatch never reads current_learnrate).
 * ---------------------------------------------------------------------------------------- */
static int64_t ora_row_len(const int64_t* off, int32_t n_rows, int32_t r) {
    return r < n_rows ? off[r + 1] - off[r] : 0;
}

void ora_socialmf_iterate(const ora_bmf_params* p, float social_reg, const int32_t* users,
                          const int32_t* items, const float* values, const int32_t* idx,
                          int64_t n_idx, int32_t n_users, int32_t n_items, const int64_t* conn_off,
                          const int32_t* conn_cols, int32_t n_conn, const int64_t* rev_off,
                          const int32_t* rev_cols, int32_t n_rev, float* U, float* V, float* bu,
                          float* bi) {
    const int k = p->k;
    float* Ug = (float*)calloc((size_t)n_users * k, sizeof(float));
    float* Vg = (float*)calloc((size_t)n_items * k, sizeof(float));
    float* bug = (float*)calloc((size_t)n_users, sizeof(float));
    float* big = (float*)calloc((size_t)n_items, sizeof(float));
    float* sum = (float*)malloc(sizeof(float) * (size_t)k);
    /* I.1 prediction error (:89-115): float score, float prediction, error = prediction - r */
    for (int64_t n = 0; n < n_idx; n++) {
        const int32_t index = idx[n];
        const int32_t u = users[index], i = items[index];
        float score = (p->global_bias + bu[u]) + bi[i];
        score += ora_row_scalar_product(U, u, V, i, k);
        const double sig = 1.0 / (1.0 + exp(-(double)score));
        const float prediction = (float)((double)p->min_rating + sig * (double)p->rating_range_size);
        const double err = (double)(prediction - values[index]);
        float g;
        if (p->loss == ORA_LOSS_MAE) {
            const double sgn = (err > 0) ? 1.0 : ((err < 0) ? -1.0 : 0.0);
            g = (float)(sgn * sig * (1.0 - sig) * (double)p->rating_range_size);
        } else if (p->loss == ORA_LOSS_LOGISTIC) {
            g = (float)err;
        } else {
            g = (float)(err * sig * (1.0 - sig) * (double)p->rating_range_size);
        }
        bug[u] += g;
        big[i] += g;
        for (int f = 0; f < k; f++) {
            Ug[(int64_t)u * k + f] += g * V[(int64_t)i * k + f];
            Vg[(int64_t)i * k + f] += g * U[(int64_t)u * k + f];
        }
    }
    /* I.2 L2 regularisation (:119-130) */
    for (int32_t u = 0; u < n_users; u++) bug[u] += bu[u] * p->reg_u * p->bias_reg;
    for (int32_t i = 0; i < n_items; i++) big[i] += bi[i] * p->reg_i * p->bias_reg;
    for (int64_t e = 0; e < (int64_t)n_users * k; e++) Ug[e] += U[e] * p->reg_u;
    for (int64_t e = 0; e < (int64_t)n_items * k; e++) Vg[e] += V[e] * p->reg_i;
    /* I.3 social regularisation, eq. (13) of the paper (:133-177) */
    if (social_reg != 0.0f)
        for (int32_t u = 0; u < n_users; u++) {
            float bias_sum = 0.0f;
            for (int f = 0; f < k; f++) sum[f] = 0.0f;
            const int64_t num = ora_row_len(conn_off, n_conn, u);
            for (int64_t x = 0; x < num; x++) {
                const int32_t v = conn_cols[conn_off[u] + x];
                bias_sum += bu[v];
                for (int f = 0; f < k; f++) sum[f] += U[(int64_t)v * k + f];
            }
            if (num != 0) {
                bug[u] += social_reg * (bu[u] - bias_sum / (float)num);
                for (int f = 0; f < k; f++)
                    Ug[(int64_t)u * k + f] +=
                        social_reg * (U[(int64_t)u * k + f] - sum[f] / (float)num);
            }
            const int64_t nrev = ora_row_len(rev_off, n_rev, u);
            for (int64_t y = 0; y < nrev; y++) {
                const int32_t v = rev_cols[rev_off[u] + y];
                const int64_t cv = ora_row_len(conn_off, n_conn, v);
                const float trust_v = 1.0f / (float)cv;
                const float neg_trust_times_reg = -social_reg * trust_v;
                float bias_diff = 0.0f;
                for (int f = 0; f < k; f++) sum[f] = 0.0f; /* factor_diffs */
                for (int64_t x = 0; x < cv; x++) {
                    const int32_t w = conn_cols[conn_off[v] + x];
                    bias_diff -= bu[w];
                    for (int f = 0; f < k; f++) sum[f] -= U[(int64_t)w * k + f];
                }
                bias_diff *= trust_v;
                bias_diff += bu[v];
                bug[u] += neg_trust_times_reg * bias_diff;
                for (int f = 0; f < k; f++) {
                    sum[f] *= trust_v;
                    sum[f] += U[(int64_t)v * k + f];
                    Ug[(int64_t)u * k + f] += neg_trust_times_reg * sum[f];
                }
            }
        }
    /* II. gradient step with LearnRate (:180-193) */
    if (p->update_user) {
        for (int32_t u = 0; u < n_users; u++)
            bu[u] -= bug[u] * p->learn_rate * p->bias_learn_rate;
        for (int64_t e = 0; e < (int64_t)n_users * k; e++) U[e] += Ug[e] * -p->learn_rate;
    }
    if (p->update_item) {
        for (int32_t i = 0; i < n_items; i++)
            bi[i] -= big[i] * p->learn_rate * p->bias_learn_rate;
        for (int64_t e = 0; e < (int64_t)n_items * k; e++) V[e] += Vg[e] * -p->learn_rate;
    }
    free(Ug);
    free(Vg);
    free(bug);
    free(big);
    free(sum);
}

/* MultiCore.PartitionUsersAndItems (MultiCore.cs:43-73).  Produces blocks as a CSR over
 * block id b = ug * G + ig: offsets[G*G+1], indices[n].  Returns G (clipped). */
int32_t ora_partition_users_and_items(ora_rng* r, const int32_t* users, const int32_t* items,
                                      int64_t n, int32_t max_user_id, int32_t max_item_id,
                                      int32_t num_groups, int64_t* offsets, int32_t* indices) {
    int32_t G = num_groups;
    if (G > max_user_id + 1) G = max_user_id + 1;
    if (G > max_item_id + 1) G = max_item_id + 1;
    int32_t* up = (int32_t*)malloc(sizeof(int32_t) * (size_t)(max_user_id + 1));
    int32_t* ip = (int32_t*)malloc(sizeof(int32_t) * (size_t)(max_item_id + 1));
    for (int32_t x = 0; x <= max_user_id; x++) up[x] = x;
    for (int32_t x = 0; x <= max_item_id; x++) ip[x] = x;
    ora_shuffle_i32(r, up, max_user_id + 1);
    ora_shuffle_i32(r, ip, max_item_id + 1);
    int64_t nb = (int64_t)G * G;
    memset(offsets, 0, sizeof(int64_t) * (size_t)(nb + 1));
    for (int64_t x = 0; x < n; x++) {
        int64_t b = (int64_t)(up[users[x]] % G) * G + (ip[items[x]] % G);
        offsets[b + 1]++;
    }
    for (int64_t b = 0; b < nb; b++) offsets[b + 1] += offsets[b];
    int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * (size_t)nb);
    memcpy(fill, offsets, sizeof(int64_t) * (size_t)nb);
    for (int64_t x = 0; x < n; x++) {
        int64_t b = (int64_t)(up[users[x]] % G) * G + (ip[items[x]] % G);
        indices[fill[b]++] = (int32_t)x;
    }
    for (int64_t b = 0; b < nb; b++)
        ora_shuffle_i32(r, indices + offsets[b], offsets[b + 1] - offsets[b]);
    free(fill);
    free(up);
    free(ip);
    return G;
}

/* BiasedMatrixFactorization.Iterate() with MaxThreads = G (:205-215): per sub-epoch i of the
 * shuffled sequence, Parallel.For over j runs block (j, (i + j) % G) -- blocks of one sub-epoch
 * share no user and no item -- on up to n_threads threads, then joins (the CPU baseline of the
 * reference's own multi-core DSGD).  Blocks as produced by ora_partition_users_and_items. */
typedef struct {
    const ora_bmf_params* p;
    const int32_t *users, *items, *idx, *cu, *ci;
    const float* values;
    const int64_t* off;
    float *U, *V, *bu, *bi;
    int32_t G, sub, t, T;
} ora_dsgd_job;

static void* ora_dsgd_worker(void* arg) {
    const ora_dsgd_job* j = (const ora_dsgd_job*)arg;
    for (int32_t x = j->t; x < j->G; x += j->T) {
        const int64_t b = (int64_t)x * j->G + (j->sub + x) % j->G;
        ora_bmf_iterate(j->p, j->users, j->items, j->values, j->idx + j->off[b],
                        j->off[b + 1] - j->off[b], j->U, j->V, j->bu, j->bi, j->cu, j->ci);
    }
    return NULL;
}

void ora_bmf_dsgd_epoch_mt(const ora_bmf_params* p, const int32_t* users, const int32_t* items,
                           const float* values, const int64_t* offsets, const int32_t* indices,
                           int32_t G, const int32_t* subepochs, int32_t n_threads, float* U,
                           float* V, float* bu, float* bi, const int32_t* count_by_user,
                           const int32_t* count_by_item) {
    if (n_threads < 1) n_threads = 1;
    if (n_threads > G) n_threads = G;
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)n_threads);
    ora_dsgd_job* jobs = (ora_dsgd_job*)malloc(sizeof(ora_dsgd_job) * (size_t)n_threads);
    for (int32_t s = 0; s < G; s++) {
        for (int32_t t = 0; t < n_threads; t++) {
            ora_dsgd_job jb = {p, users, items, indices, count_by_user, count_by_item, values,
                               offsets, U, V, bu, bi, G, subepochs[s], t, n_threads};
            jobs[t] = jb;
            pthread_create(&th[t], NULL, ora_dsgd_worker, &jobs[t]);
        }
        for (int32_t t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
    }
    free(jobs);
    free(th);
}

/* ------------------------------------------------------------------------------------------
 * BPRMF (ItemRecommendation/BPRMF.cs).  The user->items sets (SparseBooleanMatrix rows of
 * HashSet<int>) are given as a CSR in HashSet enumeration order = first-insertion order
 * (no removals), plus a per-row sorted copy for the Contains() probes.
 * ---------------------------------------------------------------------------------------- */
typedef struct {
    int32_t k;
    int32_t update_u, update_i, update_j;
    float learn_rate, reg_u, reg_i, reg_j, bias_reg;
    int32_t max_user_id, max_item_id;
    int32_t model;   /* 0 BPRMF, 1 SoftMarginRankingMF (UpdateFactors) */
    int32_t sampler; /* 0 SampleTriple of BPRMF, 2 WeightedBPRMF.SampleTriple,
                        3 IterateWithReplacementUniformUser, 4 IterateWithReplacementUniformPair */
    const int32_t* ev_users; /* Feedback.Users / Feedback.Items (event order), sampler 2 */
    const int32_t* ev_items;
    int64_t n_events;
} ora_bpr_params;

size_t ora_bpr_params_sizeof(void) { return sizeof(ora_bpr_params); }

static int ora_row_contains(const int64_t* off, const int32_t* sorted, int32_t u, int32_t item) {
    int64_t lo = off[u], hi = off[u + 1];
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (sorted[mid] < item) lo = mid + 1;
        else hi = mid;
    }
    return lo < off[u + 1] && sorted[lo] == item;
}

/* SampleUser :300-310, SampleItemPair :290-296, SampleTriple :316-321; sampler 2:
 * WeightedBPRMF.SampleTriple (ItemRecommendation/WeightedBPRMF.cs:55-67): (u, i) = the event at
 * Next(Feedback.Count), j = Feedback.Items[Next(Feedback.Count)] until j is not in S_u. */
void ora_bpr_sample_triple(ora_rng* r, const ora_bpr_params* p, const int64_t* off,
                           const int32_t* rows, const int32_t* sorted, int32_t* out) {
    if (p->sampler == 2) {
        const int32_t n = (int32_t)p->n_events;
        const int32_t index = ora_rng_next(r, n);
        const int32_t wu = p->ev_users[index], wi = p->ev_items[index];
        int32_t wj;
        do wj = p->ev_items[ora_rng_next(r, n)];
        while (ora_row_contains(off, sorted, wu, wj));
        out[0] = wu;
        out[1] = wi;
        out[2] = wj;
        return;
    }
    int32_t u;
    for (;;) {
        u = ora_rng_next(r, p->max_user_id + 1);
        int64_t cnt = (u < 0) ? 0 : off[u + 1] - off[u];
        if (cnt == 0 || cnt == (int64_t)p->max_item_id + 1) continue;
        break;
    }
    int64_t cnt = off[u + 1] - off[u];
    int32_t i = rows[off[u] + ora_rng_next(r, (int32_t)cnt)];
    int32_t j;
    do j = ora_rng_next(r, p->max_item_id + 1);
    while (ora_row_contains(off, sorted, u, j));
    out[0] = u;
    out[1] = i;
    out[2] = j;
}

/* SoftMarginRankingMF.UpdateFactors (ItemRecommendation/SoftMarginRankingMF.cs:66-113): no
 * update when x_uij > 0; otherwise the hinge gradient -- all the update expressions are float
 * arithmetic in C# (float operands, int literal 1) widened to double before the learn-rate step. */
static void ora_soft_margin_update(const ora_bpr_params* p, int32_t i, int32_t j, float* w,
                                   float* hi, float* hj, float* bias, double x_uij) {
    if (x_uij > 0) return;
    const double lr = (double)p->learn_rate;
    if (p->update_i) {
        const double bias_update = (double)(1.0f - p->bias_reg * bias[i]);
        bias[i] += (float)(lr * bias_update);
    }
    if (p->update_j) {
        const double bias_update = (double)(-1.0f - p->bias_reg * bias[j]);
        bias[j] += (float)(lr * bias_update);
    }
    for (int f = 0; f < p->k; f++) {
        const float w_uf = w[f], h_if = hi[f], h_jf = hj[f];
        if (p->update_u) {
            const double uf_update = (double)(h_if - h_jf - p->reg_u * w_uf);
            w[f] = (float)((double)w_uf + lr * uf_update);
        }
        if (p->update_i) {
            const double if_update = (double)(w_uf - p->reg_i * h_if);
            hi[f] = (float)((double)h_if + lr * if_update);
        }
        if (p->update_j) {
            const double jf_update = (double)(-w_uf - p->reg_j * h_jf);
            hj[f] = (float)((double)h_jf + lr * jf_update);
        }
    }
}

/* BPRMF.UpdateFactors(u,i,j,...) :330-374 (model 1: SoftMarginRankingMF's override) */
void ora_bpr_update(const ora_bpr_params* p, int32_t u, int32_t i, int32_t j, float* U, float* V,
                    float* bias) {
    const int k = p->k;
    float* w = U + (int64_t)u * k;
    float* hi = V + (int64_t)i * k;
    float* hj = V + (int64_t)j * k;
    double x_uij = (double)(bias[i] - bias[j]) +
                   ora_row_scalar_product_with_row_difference(U, u, V, i, V, j, k);
    if (p->model == 1) {
        ora_soft_margin_update(p, i, j, w, hi, hj, bias, x_uij);
        return;
    }
    double e = 1.0 / (1.0 + exp(x_uij));
    if (p->update_i) {
        double update = e - (double)(p->bias_reg * bias[i]);
        bias[i] += (float)((double)p->learn_rate * update);
    }
    if (p->update_j) {
        double update = -e - (double)(p->bias_reg * bias[j]);
        bias[j] += (float)((double)p->learn_rate * update);
    }
    for (int f = 0; f < k; f++) {
        float w_uf = w[f], h_if = hi[f], h_jf = hj[f];
        if (p->update_u) {
            double update = (double)(h_if - h_jf) * e - (double)(p->reg_u * w_uf);
            w[f] = (float)((double)w_uf + (double)p->learn_rate * update);
        }
        if (p->update_i) {
            double update = (double)w_uf * e - (double)(p->reg_i * h_if);
            hi[f] = (float)((double)h_if + (double)p->learn_rate * update);
        }
        if (p->update_j) {
            double update = (double)(-w_uf) * e - (double)(p->reg_j * h_jf);
            hj[f] = (float)((double)h_jf + (double)p->learn_rate * update);
        }
    }
}

/* Loss-sample burn in BPRMF.Train :136-150 (triples drawn, never used) */
void ora_bpr_burn(ora_rng* r, const ora_bpr_params* p, const int64_t* off, const int32_t* rows,
                  const int32_t* sorted, int64_t count) {
    int32_t t[3];
    for (int64_t c = 0; c < count; c++) ora_bpr_sample_triple(r, p, off, rows, sorted, t);
}

/* SampleUser :300-310 */
static int32_t ora_bpr_sample_user(ora_rng* r, const ora_bpr_params* p, const int64_t* off) {
    for (;;) {
        int32_t u = ora_rng_next(r, p->max_user_id + 1);
        int64_t cnt = off[u + 1] - off[u];
        if (cnt == 0 || cnt == (int64_t)p->max_item_id + 1) continue;
        return u;
    }
}

/* One epoch of num_events triples, each sampled then applied; if trace != NULL the triples are
 * recorded (3 * num_events ints).
 *   sampler 0 / 2: IterateWithoutReplacementUniformUser :216-226 (SampleTriple per event)
 *   sampler 3: IterateWithReplacementUniformUser :183-211.  user_matrix = GetUserMatrixCopy()
 *     (Data/PosOnlyFeedback.cs:68-74) once per epoch: each row a HashSet filled in event order.
 *     ElementAt(Next(Count)) enumerates the set's slots in index order and Remove (the `= false`
 *     setter) frees one slot without moving the others, so the remaining items keep their insertion
 *     order; removing the last one leaves an empty set (count 0, lastIndex 0), which the reset at
 *     :198-200 refills with Feedback.UserMatrix[u] in its enumeration order -- the full row again.
 *     The negative is drawn against the full set, Feedback.UserMatrix[u] (:204-206).
 *   sampler 4: IterateWithReplacementUniformPair :231-243: the event at Next(Count), then
 *     SampleOtherItem :275-284 (the given item is positive, so j is redrawn while in S_u). */
void ora_bpr_epoch(ora_rng* r, const ora_bpr_params* p, const int64_t* off, const int32_t* rows,
                   const int32_t* sorted, int64_t num_events, float* U, float* V, float* bias,
                   int32_t* trace) {
    int32_t t[3];
    int32_t* rem = NULL;  /* sampler 3: each user's remaining items, insertion order */
    int64_t* left = NULL; /* sampler 3: how many remain */
    if (p->sampler == 3) {
        const int64_t n_rows = (int64_t)p->max_user_id + 1, nnz = off[n_rows];
        rem = (int32_t*)malloc(sizeof(int32_t) * (size_t)(nnz > 0 ? nnz : 1));
        left = (int64_t*)malloc(sizeof(int64_t) * (size_t)n_rows);
        memcpy(rem, rows, sizeof(int32_t) * (size_t)nnz);
        for (int64_t u = 0; u < n_rows; u++) left[u] = off[u + 1] - off[u];
    }
    for (int64_t c = 0; c < num_events; c++) {
        if (p->sampler == 3) {
            const int32_t u = ora_bpr_sample_user(r, p, off);
            int32_t* row = rem + off[u];
            if (left[u] == 0) { /* reset: refill from Feedback.UserMatrix[u] */
                left[u] = off[u + 1] - off[u];
                memcpy(row, rows + off[u], sizeof(int32_t) * (size_t)left[u]);
            }
            const int32_t x = ora_rng_next(r, (int32_t)left[u]);
            const int32_t i = row[x];
            memmove(row + x, row + x + 1, sizeof(int32_t) * (size_t)(left[u] - x - 1));
            left[u]--;
            int32_t j;
            do j = ora_rng_next(r, p->max_item_id + 1);
            while (ora_row_contains(off, sorted, u, j));
            t[0] = u;
            t[1] = i;
            t[2] = j;
        } else if (p->sampler == 4) {
            const int32_t index = ora_rng_next(r, (int32_t)p->n_events);
            const int32_t u = p->ev_users[index], i = p->ev_items[index];
            const int item_is_positive = ora_row_contains(off, sorted, u, i);
            int32_t j;
            do j = ora_rng_next(r, p->max_item_id + 1);
            while (ora_row_contains(off, sorted, u, j) == item_is_positive);
            t[0] = u;
            t[1] = i;
            t[2] = j;
        } else {
            ora_bpr_sample_triple(r, p, off, rows, sorted, t);
        }
        if (trace) {
            trace[3 * c] = t[0];
            trace[3 * c + 1] = t[1];
            trace[3 * c + 2] = t[2];
        }
        ora_bpr_update(p, t[0], t[1], t[2], U, V, bias);
    }
    free(rem);
    free(left);
}

/* ------------------------------------------------------------------------------------------
 * Large-set drivers of the same arithmetic (C3-density checks).  Both produce exactly what the
 * sequential loops above produce: the sampler draws from the RNG in the same order and
 * UpdateFactors runs over the same triples in the same order.  They only overlap the memory
 * latency of a 1 M x 1 M set -- triples do not depend on the factors (BPRMF.cs:216-226), so the
 * sampler can run ahead of the updates, and the rows of the next triples can be prefetched.
 * ---------------------------------------------------------------------------------------- */
#define ORA_AHEAD 8

static void ora_bpr_prefetch(const ora_bpr_params* p, const int32_t* t, const float* U,
                             const float* V) {
    const int64_t k = p->k;
    for (int64_t f = 0; f < k; f += 16) {
        __builtin_prefetch(U + (int64_t)t[0] * k + f, 1);
        __builtin_prefetch(V + (int64_t)t[1] * k + f, 1);
        __builtin_prefetch(V + (int64_t)t[2] * k + f, 1);
    }
}

/* UpdateFactors over given triples in order (a replay of a recorded triple stream) */
void ora_bpr_apply_triples(const ora_bpr_params* p, const int32_t* tu, const int32_t* ti,
                           const int32_t* tj, int64_t n, float* U, float* V, float* bias) {
    for (int64_t c = 0; c < n; c++) {
        if (c + ORA_AHEAD < n) {
            const int32_t t[3] = {tu[c + ORA_AHEAD], ti[c + ORA_AHEAD], tj[c + ORA_AHEAD]};
            ora_bpr_prefetch(p, t, U, V);
        }
        ora_bpr_update(p, tu[c], ti[c], tj[c], U, V, bias);
    }
}

#define ORA_RING (1 << 16)
typedef struct {
    ora_rng* r;
    const ora_bpr_params* p;
    const int64_t *off;
    const int32_t *rows, *sorted;
    int64_t n;
    int32_t* ring; /* 3 * ORA_RING */
    _Atomic int64_t head, tail;
} ora_bpr_pipe;

static void* ora_bpr_producer(void* arg) {
    ora_bpr_pipe* q = (ora_bpr_pipe*)arg;
    for (int64_t c = 0; c < q->n; c++) {
        while (c - atomic_load_explicit(&q->tail, memory_order_acquire) >= ORA_RING) {
        }
        ora_bpr_sample_triple(q->r, q->p, q->off, q->rows, q->sorted, q->ring + 3 * (c % ORA_RING));
        atomic_store_explicit(&q->head, c + 1, memory_order_release);
    }
    return NULL;
}

/* ora_bpr_epoch for the default sampler (SampleTriple per event, :216-226): one thread samples,
 * the caller applies UpdateFactors in sample order, ORA_AHEAD triples' rows prefetched */
void ora_bpr_epoch_pipelined(ora_rng* r, const ora_bpr_params* p, const int64_t* off,
                             const int32_t* rows, const int32_t* sorted, int64_t num_events,
                             float* U, float* V, float* bias, int32_t* trace) {
    if (p->sampler != 0) {
        ora_bpr_epoch(r, p, off, rows, sorted, num_events, U, V, bias, trace);
        return;
    }
    ora_bpr_pipe* q = (ora_bpr_pipe*)calloc(1, sizeof(ora_bpr_pipe));
    q->r = r;
    q->p = p;
    q->off = off;
    q->rows = rows;
    q->sorted = sorted;
    q->n = num_events;
    q->ring = (int32_t*)malloc(sizeof(int32_t) * 3 * ORA_RING);
    atomic_init(&q->head, 0);
    atomic_init(&q->tail, 0);
    pthread_t th;
    pthread_create(&th, NULL, ora_bpr_producer, q);
    for (int64_t c = 0; c < num_events; c++) {
        int64_t h;
        while ((h = atomic_load_explicit(&q->head, memory_order_acquire)) <= c) {
        }
        if (c + ORA_AHEAD < h) ora_bpr_prefetch(p, q->ring + 3 * ((c + ORA_AHEAD) % ORA_RING), U, V);
        const int32_t* t = q->ring + 3 * (c % ORA_RING);
        if (trace) {
            trace[3 * c] = t[0];
            trace[3 * c + 1] = t[1];
            trace[3 * c + 2] = t[2];
        }
        ora_bpr_update(p, t[0], t[1], t[2], U, V, bias);
        atomic_store_explicit(&q->tail, c + 1, memory_order_release);
    }
    pthread_join(th, NULL);
    free(q->ring);
    free(q);
}

/* transparent huge pages for a large array before it is first written (fewer TLB misses on the
 * random row accesses of the large-set drivers); advice only, no effect on any value */
int ora_madvise_huge(void* ptr, int64_t bytes) {
    const uintptr_t a = ((uintptr_t)ptr + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1);
    const uintptr_t e = ((uintptr_t)ptr + (uintptr_t)bytes) & ~(uintptr_t)((2u << 20) - 1);
    if (e <= a) return 0;
    return madvise((void*)a, e - a, MADV_HUGEPAGE);
}

/* ------------------------------------------------------------------------------------------
 * WRMF (ItemRecommendation/WRMF.cs:79-156), fp64.  One half-step: W rows from H.
 * data rows as CSR (insertion order).  Inverse via LU with partial pivoting, like MathNet's
 * DenseMatrix.Inverse() (managed provider).
 * ---------------------------------------------------------------------------------------- */
static void ora_lu_inverse(double* a, double* inv, int n, int* piv, double* col) {
    /* LU factorisation in place with partial pivoting (row interchanges) */
    for (int i = 0; i < n; i++) piv[i] = i;
    for (int c = 0; c < n; c++) {
        int p = c;
        double best = fabs(a[c * n + c]);
        for (int r = c + 1; r < n; r++)
            if (fabs(a[r * n + c]) > best) {
                best = fabs(a[r * n + c]);
                p = r;
            }
        if (p != c) {
            for (int x = 0; x < n; x++) {
                double t = a[c * n + x];
                a[c * n + x] = a[p * n + x];
                a[p * n + x] = t;
            }
            int t = piv[c];
            piv[c] = piv[p];
            piv[p] = t;
        }
        double d = a[c * n + c];
        if (d != 0.0)
            for (int r = c + 1; r < n; r++) {
                a[r * n + c] /= d;
                double m = a[r * n + c];
                for (int x = c + 1; x < n; x++) a[r * n + x] -= m * a[c * n + x];
            }
    }
    /* solve A X = I column by column */
    for (int j = 0; j < n; j++) {
        for (int i = 0; i < n; i++) col[i] = (piv[i] == j) ? 1.0 : 0.0;
        for (int i = 0; i < n; i++) {
            double s = col[i];
            for (int x = 0; x < i; x++) s -= a[i * n + x] * col[x];
            col[i] = s;
        }
        for (int i = n - 1; i >= 0; i--) {
            double s = col[i];
            for (int x = i + 1; x < n; x++) s -= a[i * n + x] * col[x];
            col[i] = s / a[i * n + i];
        }
        for (int i = 0; i < n; i++) inv[i * n + j] = col[i];
    }
}

/* WRMF.ComputeSquareMatrix :94-108 -- float products, double sums */
void ora_wrmf_square(const float* H, int64_t rows, int k, double* HH) {
    for (int f1 = 0; f1 < k; f1++)
        for (int f2 = f1; f2 < k; f2++) {
            double d = 0.0;
            for (int64_t i = 0; i < rows; i++) d += (double)(H[i * k + f1] * H[i * k + f2]);
            HH[f1 * k + f2] = d;
            HH[f2 * k + f1] = d;
        }
}

/* WRMF.Optimize(u, data, W, H, HH) :110-156 over rows [row_begin, row_end).  exact = 0: the
 * reference's arithmetic -- each product h[f1] * h[f2] of the row Gram rounded to float before its
 * double sum (:116-121).  exact = 1 (test infrastructure, not a reference function): the same
 * system with those products exact in double, (double) h[f1] * (double) h[f2]; HH (the caller's,
 * ComputeSquareMatrix's float products) and everything else unchanged.  That is the system an
 * fp64 solver with an exact residual lands on (the library's Precision = fp64 mode), so it pins
 * the refinement independently of the float-product floor. */
static void wrmf_optimize_rows_impl(const int64_t* off, const int32_t* cols, int64_t row_begin,
                                    int64_t row_end, int64_t n_data_rows, float* W,
                                    const float* H, const double* HH, int k, double alpha,
                                    double reg, int exact);

void ora_wrmf_optimize_rows(const int64_t* off, const int32_t* cols, int64_t row_begin,
                            int64_t row_end, int64_t n_data_rows, float* W, const float* H,
                            const double* HH, int k, double alpha, double reg) {
    wrmf_optimize_rows_impl(off, cols, row_begin, row_end, n_data_rows, W, H, HH, k, alpha, reg,
                            0);
}

void ora_wrmf_optimize_rows_exact(const int64_t* off, const int32_t* cols, int64_t row_begin,
                                  int64_t row_end, int64_t n_data_rows, float* W, const float* H,
                                  const double* HH, int k, double alpha, double reg) {
    wrmf_optimize_rows_impl(off, cols, row_begin, row_end, n_data_rows, W, H, HH, k, alpha, reg,
                            1);
}

static void wrmf_optimize_rows_impl(const int64_t* off, const int32_t* cols, int64_t row_begin,
                                    int64_t row_end, int64_t n_data_rows, float* W,
                                    const float* H, const double* HH, int k, double alpha,
                                    double reg, int exact) {
    double* HC = (double*)malloc(sizeof(double) * (size_t)k * k);
    double* m = (double*)malloc(sizeof(double) * (size_t)k * k);
    double* inv = (double*)malloc(sizeof(double) * (size_t)k * k);
    double* HCp = (double*)malloc(sizeof(double) * (size_t)k);
    double* col = (double*)malloc(sizeof(double) * (size_t)k);
    int* piv = (int*)malloc(sizeof(int) * (size_t)k);
    for (int64_t u = row_begin; u < row_end; u++) {
        int64_t b = (u < n_data_rows) ? off[u] : 0, e = (u < n_data_rows) ? off[u + 1] : 0;
        for (int f1 = 0; f1 < k; f1++)
            for (int f2 = f1; f2 < k; f2++) {
                double d = 0.0;
                for (int64_t x = b; x < e; x++) {
                    const float* h = H + (int64_t)cols[x] * k;
                    d += exact ? (double)h[f1] * (double)h[f2] : (double)(h[f1] * h[f2]);
                }
                HC[f1 * k + f2] = d * alpha;
                HC[f2 * k + f1] = d * alpha;
            }
        for (int f = 0; f < k; f++) {
            double d = 0.0;
            for (int64_t x = b; x < e; x++) d += (double)H[(int64_t)cols[x] * k + f];
            HCp[f] = d * (1.0 + alpha);
        }
        for (int f1 = 0; f1 < k; f1++)
            for (int f2 = f1; f2 < k; f2++) {
                double d = HH[f1 * k + f2] + HC[f1 * k + f2];
                if (f1 == f2) d += reg;
                m[f1 * k + f2] = d;
                m[f2 * k + f1] = d;
            }
        ora_lu_inverse(m, inv, k, piv, col);
        for (int f = 0; f < k; f++) {
            double d = 0.0;
            for (int f2 = 0; f2 < k; f2++) d += inv[f * k + f2] * HCp[f2];
            W[u * k + f] = (float)d;
        }
    }
    free(HC);
    free(m);
    free(inv);
    free(HCp);
    free(col);
    free(piv);
}

/* ------------------------------------------------------------------------------------------
 * Item-recommendation evaluation: Eval/Items.cs:126-209 + AUC.Compute (Eval/Measures/AUC.cs:42-68)
 * for an MF-style scorer score(u,i) = bias[i] + <U_u, V_i> (bias may be NULL: MF.Predict).
 * candidates: already-shuffled candidate list (Items.Candidates :62-96).
 * train/test user rows as CSR.  Returns AUC averaged with float accumulation; *num_users out.
 * ---------------------------------------------------------------------------------------- */
typedef struct {
    float score;
    int32_t pos;
    int32_t item;
} ora_scored;

static int ora_cmp_scored(const void* a, const void* b) {
    const ora_scored* x = (const ora_scored*)a;
    const ora_scored* y = (const ora_scored*)b;
    if (x->score > y->score) return -1; /* descending */
    if (x->score < y->score) return 1;
    return (x->pos < y->pos) ? -1 : (x->pos > y->pos); /* OrderByDescending is stable */
}

/* AUC.Compute with rank list given implicitly (relevance flags in ranked order) */
double ora_auc_compute(const int32_t* ranked_relevant, int64_t n_ranked, int64_t n_relevant_total,
                       int64_t num_dropped_items) {
    int64_t num_relevant_in_list = 0;
    for (int64_t x = 0; x < n_ranked; x++) num_relevant_in_list += ranked_relevant[x] ? 1 : 0;
    int64_t num_eval_items = n_ranked + num_dropped_items;
    int64_t num_eval_pairs = (num_eval_items - num_relevant_in_list) * num_relevant_in_list;
    if (num_eval_pairs < 0) return -1.0;
    if (num_eval_pairs == 0) return 0.5;
    int64_t correct = 0, hit = 0;
    for (int64_t x = 0; x < n_ranked; x++) {
        if (!ranked_relevant[x]) correct += hit;
        else hit++;
    }
    int64_t missing = n_relevant_total - num_relevant_in_list;
    correct += hit * (num_dropped_items - missing);
    return (double)correct / (double)num_eval_pairs;
}

float ora_item_eval_auc(const int32_t* test_users, int64_t n_test_users, const int32_t* candidates,
                        int64_t n_cand, const int64_t* tr_off, const int32_t* tr_cols,
                        int64_t tr_rows, const int64_t* te_off, const int32_t* te_cols,
                        int64_t te_rows, int32_t n_items_total, int32_t max_user_id,
                        int32_t max_item_id, int k, const float* U, const float* V,
                        const float* bias, int32_t* num_users_out) {
    uint8_t* is_cand = (uint8_t*)calloc((size_t)n_items_total, 1);
    uint8_t* is_correct = (uint8_t*)calloc((size_t)n_items_total, 1);
    uint8_t* is_ignored = (uint8_t*)calloc((size_t)n_items_total, 1);
    ora_scored* buf = (ora_scored*)malloc(sizeof(ora_scored) * (size_t)(n_cand + 1));
    int32_t* flags = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n_cand + 1));
    for (int64_t c = 0; c < n_cand; c++) is_cand[candidates[c]] = 1;
    float auc_sum = 0.0f;
    int32_t num_users = 0;
    for (int64_t t = 0; t < n_test_users; t++) {
        int32_t u = test_users[t];
        int64_t n_correct = 0, n_ignored = 0;
        if (u < te_rows)
            for (int64_t x = te_off[u]; x < te_off[u + 1]; x++) {
                int32_t it = te_cols[x];
                if (is_cand[it] && !is_correct[it]) {
                    is_correct[it] = 1;
                    n_correct++;
                }
            }
        if (u < tr_rows)
            for (int64_t x = tr_off[u]; x < tr_off[u + 1]; x++) {
                int32_t it = tr_cols[x];
                if (is_cand[it] && !is_ignored[it]) {
                    is_ignored[it] = 1;
                    n_ignored++;
                }
            }
        int skip = (n_correct == 0) || (n_correct == n_cand - n_ignored);
        if (!skip) {
            int64_t m = 0;
            for (int64_t c = 0; c < n_cand; c++) {
                int32_t it = candidates[c];
                if (is_ignored[it]) continue;
                float s;
                if (u > max_user_id || it > max_item_id) s = -3.402823466e+38f; /* float.MinValue */
                else {
                    s = ora_row_scalar_product(U, u, V, it, k);
                    if (bias) s = bias[it] + s;
                }
                if (s > -3.402823466e+38f) {
                    buf[m].score = s;
                    buf[m].pos = (int32_t)c;
                    buf[m].item = it;
                    m++;
                }
            }
            qsort(buf, (size_t)m, sizeof(ora_scored), ora_cmp_scored);
            for (int64_t x = 0; x < m; x++) flags[x] = is_correct[buf[x].item];
            int64_t num_dropped = (n_cand - n_ignored) - m;
            double auc = ora_auc_compute(flags, m, n_correct, num_dropped);
            num_users++;
            auc_sum += (float)auc;
        }
        if (u < te_rows)
            for (int64_t x = te_off[u]; x < te_off[u + 1]; x++) is_correct[te_cols[x]] = 0;
        if (u < tr_rows)
            for (int64_t x = tr_off[u]; x < tr_off[u + 1]; x++) is_ignored[tr_cols[x]] = 0;
    }
    free(is_cand);
    free(is_correct);
    free(is_ignored);
    free(buf);
    free(flags);
    *num_users_out = num_users;
    return num_users ? auc_sum / (float)num_users : 0.0f;
}
