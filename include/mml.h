/*
 * mml.h -- C ABI of libmml_hip.so, the MI355X-native training path for MyMediaLite's
 * BiasedMatrixFactorization (explicit SGD), BPRMF (pairwise SGD) and WRMF (implicit ALS).
 *
 * Drop-in boundary.  The reference has no native code and no C ABI: these
 * entry points are what the C# front end binds through P/Invoke to replace
 * the managed inner loops named next to each function.  Conventions:
 *   - every call returns mml_status (0 = OK, < 0 = error class); the message of the last failed
 *     call on this host thread is mml_last_error().  A failure never aborts the host process.
 *   - all arrays are plain host pointers unless the name says _device; the library COPIES host
 *     buffers into HBM it owns and retains no caller pointer after a call returns.
 *   - calls on one handle must come from one host thread at a time; every call is synchronous
 *     (an epoch has finished when mml_*_iterate returns), preserving IIterativeModel.Iterate().
 *   - row-major float factor matrices, exactly Matrix<float>.data
 *     (src/MyMediaLite/DataType/Matrix.cs:29-36, element (i,j) at data[i*dim2+j]).
 */
#ifndef MML_H
#define MML_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MML_ABI_VERSION 14

typedef int32_t mml_status;
enum {
    MML_OK = 0,
    MML_ERR_ARG = -1,     /* bad argument (null pointer, size, id out of range) */
    MML_ERR_HIP = -2,     /* HIP runtime error */
    MML_ERR_RCCL = -3,    /* RCCL error */
    MML_ERR_OOM = -4,     /* device allocation failed */
    MML_ERR_STATE = -5,   /* call not valid in the handle's current state */
    MML_ERR_NODEV = -6    /* no usable gfx950 device */
};

/* ------------------------------------------------------------------ library / context */
int mml_abi_version(void);
const char* mml_last_error(void);
mml_status mml_device_count(int32_t* out);

typedef struct mml_ctx mml_ctx;
/* One context per recommender instance, bound to one GPU (one process per GPU for multi-GPU). */
mml_status mml_ctx_create(int32_t device_id, mml_ctx** out);
mml_status mml_ctx_destroy(mml_ctx* ctx);
/* One context over n GPUs driven from ONE process (ABI 4) -- the shape of the reference's
 * single-process front end (RatingPrediction.cs:161-331): an ncclCommInitAll communicator, one
 * stream per device.  Handles created on it shard the work over the devices: mml_bmf / mml_bpr
 * on the HOGWILD schedules split the ratings into user ranges of equal rating count and average
 * V || item biases with one RCCL all-reduce after every epoch; mml_bmf on the DSGD
 * schedule runs the reference's MaxThreads = G blocks (BiasedMatrixFactorization.cs:205-215) as a
 * ring: device d is rank d, owns block rows [d G/n, (d+1) G/n), item groups move by ncclSend /
 * ncclRecv to the rank whose rows visit them next, and the model equals the single-device DSGD
 * model bit for bit (G must be a multiple of n; round 4: the same rank code runs one process per
 * GPU, a one-device context with mml_ctx_comm_init, DSGD schedule, every rank given the whole
 * rating set and the same blocks and sub-epoch sequence, get_model / predict / evaluate then
 * collectives); mml_wrmf solves row shards and all-gathers them after each
 * half-step.  Each call returns when all devices have finished.  mml_bmf's user shards also run
 * the ORDERED schedule (ABI 6: each shard its own range in visit order, deterministic), and
 * mml_bmf_set_data_device takes arrays on the first listed device and shards them there (ABI 6).
 * The sibling-model extras return MML_ERR_STATE.  A device id may be listed more than once
 * (several shards on one GPU, e.g. to emulate N devices on one): such a context has no
 * communicator; mml_bmf and mml_bpr then run the shards one after another and average V || item
 * biases with peer copies and a device kernel (sum in shard order, then / N), the DSGD ring moves
 * its groups by peer copy, and mml_wrmf runs its row shards on one host thread each, all-gathering
 * by peer copies between host barriers (ABI 9).  mml_bpr's user shards also run the ORDERED
 * schedule (ABI 9), and mml_wrmf's shards take every refinement decision on the max over the
 * shards' corrections (ABI 9), so a row-sharded WRMF model equals the one-device model bit for
 * bit at any shard count, over RCCL or peer copies. */
mml_status mml_ctx_create_multi(const int32_t* device_ids, int32_t n_devices, mml_ctx** out);
/* RCCL communicator across processes (one rank per GPU): rank 0 creates the 128-byte id, the host
 * broadcasts it (e.g. torch.distributed / MPI), then every rank calls mml_ctx_comm_init. */
mml_status mml_comm_unique_id(uint8_t out_id[128]);
mml_status mml_ctx_comm_init(mml_ctx* ctx, const uint8_t id[128], int32_t nranks, int32_t rank);
/* Item groups the Hogwild schedules split the stream into (ABI 4): 8 when the device deals the
 * blocks of a grid round-robin over its 8 XCDs (probed once per context by reading each block's
 * XCC id), so each group's item rows are only cached in one XCD's L2; else 1.  No reference
 * counterpart (the managed Hogwild has one coherent cache hierarchy). */
mml_status mml_ctx_xcd_groups(mml_ctx* ctx, int32_t* out);

/* ------------------------------------------------------------------ host RNG (MyMediaLite.Random)
 * System.Random(seed)-compatible generator for hosts without the .NET BCL; the C# front end keeps
 * using its own MyMediaLite.Random (src/MyMediaLite/Random.cs:23-64) and never needs these. */
typedef struct mml_random mml_random;
mml_status mml_random_create(int32_t seed, mml_random** out);
mml_status mml_random_destroy(mml_random* r);
mml_status mml_random_next(mml_random* r, int32_t max_value, int32_t* out);   /* Random.Next(n) */
mml_status mml_random_next_double(mml_random* r, double* out);               /* NextDouble() */
/* MatrixExtensions.InitNormal (DataType/MatrixExtensions.cs:62-69): MathNet polar Normal */
mml_status mml_random_fill_normal(mml_random* r, double mean, double stddev, float* out, int64_t n);
/* Utils.Shuffle (src/MyMediaLite/Utils.cs:52-64) */
mml_status mml_random_shuffle_i32(mml_random* r, int32_t* a, int64_t n);
/* MultiCore.PartitionUsersAndItems (src/MyMediaLite/MultiCore.cs:43-73): blocks as CSR over
 * b = user_group*G + item_group; offsets[G*G+1], indices[n]; *out_groups = clipped G. */
mml_status mml_partition_users_and_items(mml_random* r, const int32_t* users, const int32_t* items,
                                         int64_t n, int32_t max_user_id, int32_t max_item_id,
                                         int32_t num_groups, int64_t* offsets, int32_t* indices,
                                         int32_t* out_groups);

/* Row shards for one process per GPU (WRMF): contiguous ranges [bounds[r],
 * bounds[r+1]) of n rows with balanced work (row weight = deg + k/2); bounds[parts + 1].
 * Host-only; every rank derives the same shards from the same degrees. */
mml_status mml_balanced_rows(const int64_t* deg, int64_t n, int32_t k, int32_t parts,
                             int64_t* bounds);

/* ------------------------------------------------------------------ rating files (host) */
/* IO/StaticRatingData.Read (src/MyMediaLite/IO/StaticRatingData.cs:36-117), multi-threaded:
 * StreamReader.ReadLine lines ("\n", "\r" or "\r\n"; a UTF-8 BOM dropped), empty lines skipped,
 * String.Split on '\t' ' ' ',' (>= 3 tokens), ids by IdentityMapping (int.Parse) or
 * Mapping.ToInternalID (first-appearance order, Data/Mapping.cs:75-85) seeded with the ids the
 * caller's mapping already holds, ratings by float.Parse.  WITHOUT_RATINGS: the
 * TestRatingFileFormat.WITHOUT_RATINGS variant (>= 2 tokens, rating 0).  ITEM_DATA: ItemData.Read
 * (IO/ItemData.cs:59-94): >= 2 tokens, lines that Trim() to nothing skipped, values all 0. */
enum {
    MML_READ_IGNORE_FIRST_LINE = 1,
    MML_READ_USER_IDENTITY = 2, /* IdentityMapping for users (else Mapping) */
    MML_READ_ITEM_IDENTITY = 4,
    MML_READ_WITHOUT_RATINGS = 8,
    MML_READ_ITEM_DATA = 16,
    /* ABI 4: the binary cache of FileSerializer (IO/FileSerializer.cs:34-77): only when both
     * columns use IdentityMapping (FileSerializer.Should), the parse result is kept next to the file
     * as <path>.bin.mml.StaticRatings (ItemData: .bin.mml.PosOnlyFeedback) -- the library's own
     * format, not BinaryFormatter's -- and a later read with the same flags loads it instead of
     * parsing (the reference loads its cache whatever the flags; here they must match, else the
     * text is parsed and the cache rewritten).  A cache that cannot be written is skipped. */
    MML_READ_BINARY_CACHE = 32,
};
typedef struct mml_rating_file mml_rating_file;
mml_status mml_rating_file_read(const char* path, int32_t flags, int32_t n_threads,
                                const char* const* user_seed, int32_t n_user_seed,
                                const char* const* item_seed, int32_t n_item_seed,
                                mml_rating_file** out);
/* n_ratings = entries; n_lines = StaticRatings size (the array length the reference allocates);
 * n_new_* = external ids the seeded mappings did not hold (internal ids n_seed, n_seed + 1, ...) */
mml_status mml_rating_file_counts(mml_rating_file* f, int64_t* n_ratings, int64_t* n_lines,
                                  int32_t* n_new_users, int32_t* n_new_items);
mml_status mml_rating_file_get(mml_rating_file* f, int32_t* users, int32_t* items, float* values);
/* which = 0 users, 1 items: all new external ids in internal-id order, each followed by '\n';
 * *bytes = their total length (cap 0: query only) */
mml_status mml_rating_file_new_ids(mml_rating_file* f, int32_t which, char* buf, int64_t cap,
                                   int64_t* bytes);
mml_status mml_rating_file_destroy(mml_rating_file* f);
/* ABI 7: the same read with the arrays landing in `ctx`'s HBM.  The file's bytes are copied to the
 * device once and tokenised there (StaticRatingData.Read's rules as above; Mapping columns resolved
 * on the device in first-appearance order when every id and seed is a canonical decimal, "0" or
 * [1-9][0-9]{0,17}; ratings on the correctly rounded fast path: <= 2^24 significant value, decimal
 * exponent within +-10).  Anything else -- ITEM_DATA, BINARY_CACHE, other id or rating spellings,
 * a malformed line -- runs mml_rating_file_read and uploads its arrays: same result and error text
 * either way.  counts / get (a device-to-host copy) / new_ids work as for a host read. */
mml_status mml_rating_file_read_device(mml_ctx* ctx, const char* path, int32_t flags,
                                       int32_t n_threads, const char* const* user_seed,
                                       int32_t n_user_seed, const char* const* item_seed,
                                       int32_t n_item_seed, mml_rating_file** out);
/* Device pointers of a read_device result (owned by f, valid until destroy; pass them to
 * mml_bmf_set_data_device etc.); *device_parsed = 1 when the device tokenised the file, 0 when the
 * host reader ran. */
mml_status mml_rating_file_device_arrays(mml_rating_file* f, const int32_t** users,
                                         const int32_t** items, const float** values,
                                         int32_t* device_parsed);

/* ------------------------------------------------------------------ BiasedMatrixFactorization */
enum { MML_LOSS_RMSE = 0, MML_LOSS_MAE = 1, MML_LOSS_LOGISTIC = 2 }; /* OptimizationTarget */
enum {
    MML_SCHEDULE_ORDERED = 0, /* exact reference order (MaxThreads = 1): one wavefront */
    MML_SCHEDULE_DSGD = 1,    /* reference DSGD (MaxThreads = G > 1): conflict-free blocks */
    MML_SCHEDULE_HOGWILD = 2, /* lock-free parallel SGD over the fixed permuted stream */
    MML_SCHEDULE_HOGWILD_COHERENT = 3 /* Hogwild with agent-coherent (sc1) row accesses: no per-XCD
                                         cache replicas of hot rows; slower on skewed items */
};

/* Model family of an mml_bmf handle. */
enum {
    MML_MF_BIASED = 0, /* BiasedMatrixFactorization (BiasedMatrixFactorization.cs:77-562) */
    MML_MF_PLAIN = 1,  /* MatrixFactorization (MatrixFactorization.cs:50-418): no biases, score =
                          global_bias + <U_u, V_i>, err = r - score in float, Regularization for
                          both sides (pass it as reg_u = reg_i), Predict clipped to [min, max];
                          loss, frequency_regularization and the bias fields are ignored and
                          mml_bmf_objective is not defined */
    MML_MF_SOCIAL = 2, /* SocialMF (SocialMF.cs:43-254): BiasedMatrixFactorization trained by
                          full-batch gradient descent with a social-network regulariser
                          (IterateBatch :77-194) over the user relation of
                          mml_bmf_set_user_relation; mml_bmf_iterate's learn_rate is LearnRate
                          (the batch step never reads current_learnrate); the schedule field is
                          ignored (the batch step is order-independent up to the per-row
                          accumulation order, which follows the stored visit order) */
    MML_MF_ITEM_ASYM = 3, /* SigmoidItemAsymmetricFactorModel (SigmoidItemAsymmetricFactorModel.cs:
                            43-344): a BiasedMatrixFactorization whose user vector is y summed over
                            the items the user rated (training + AdditionalFeedback) / sqrt(count);
                            mml_bmf_set_implicit_feedback before iterate; ORDERED (bit-faithful)
                            or HOGWILD (ABI 3) */
    MML_MF_USER_ASYM = 4, /* SigmoidUserAsymmetricFactorModel (SigmoidUserAsymmetricFactorModel.cs:
                            43-309): the mirror -- the item vector is x summed over the users who
                            rated the item / sqrt(count), each rating trains U_u and those x rows
                            (ABI 3) */
    MML_MF_COMBINED_ASYM = 5, /* SigmoidCombinedAsymmetricFactorModel
                            (SigmoidCombinedAsymmetricFactorModel.cs:46-382): both -- user vector
                            from y, item vector from x, each rating trains those x and y rows
                            (ABI 3) */
    MML_MF_SVDPP = 6,    /* SVDPlusPlus (SVDPlusPlus.cs:43-423): a MatrixFactorization with biases;
                            user vector = y summed over the user's items / sqrt(count) + p_u;
                            Predict without sigmoid, clipped (ABI 3) */
    MML_MF_SIGMOID_SVDPP = 7 /* SigmoidSVDPlusPlus (SigmoidSVDPlusPlus.cs:42-269): the same with
                            the sigmoid link and the loss variants (ABI 3) */
};

typedef struct {
    int32_t num_factors;              /* NumFactors (MatrixFactorization.cs:71) */
    int32_t loss;                     /* Loss, MML_LOSS_* (BiasedMatrixFactorization.cs:114) */
    int32_t frequency_regularization; /* FrequencyRegularization (:111) */
    int32_t schedule;                 /* MML_SCHEDULE_* */
    float bias_learn_rate;            /* BiasLearnRate (:85) */
    float bias_reg;                   /* BiasReg (:88) */
    float reg_u;                      /* RegU (:91) */
    float reg_i;                      /* RegI (:94) */
    int32_t model;                    /* MML_MF_* (ABI 2) */
    float social_regularization;      /* SocialRegularization (SocialMF.cs:46), MML_MF_SOCIAL */
} mml_bmf_params;

typedef struct mml_bmf mml_bmf;

mml_status mml_bmf_create(mml_ctx* ctx, const mml_bmf_params* params, int32_t n_users,
                          int32_t n_items, mml_bmf** out);
mml_status mml_bmf_destroy(mml_bmf* h);
/* Training ratings (StaticRatings SoA: Data/StaticRatings.cs:49-51) + the epoch visiting order:
 * order = DataSet.RandomIndex (Data/DataSet.cs:100-110), reused every epoch like the reference;
 * NULL = identity.  The device keeps the ratings permuted into visit order (coalesced stream). */
mml_status mml_bmf_set_data(mml_bmf* h, const int32_t* users, const int32_t* items,
                            const float* values, int64_t n, const int32_t* order);
/* Same, from arrays already resident in this context's HBM (device pointers).  The call first waits
 * for the work queued on the device, so the arrays may be produced on any stream. */
mml_status mml_bmf_set_data_device(mml_bmf* h, const int32_t* users_device,
                                   const int32_t* items_device, const float* values_device,
                                   int64_t n, const int32_t* order_device);
/* DSGD blocks (MML_SCHEDULE_DSGD): CSR over b = user_group*G + item_group of rating indices,
 * as produced by MultiCore.PartitionUsersAndItems / mml_partition_users_and_items.  On a
 * multi-device context the indices address the arrays given to mml_bmf_set_data, and the call
 * deals the block rows out to the devices. */
mml_status mml_bmf_set_blocks(mml_bmf* h, int32_t num_groups, const int64_t* offsets,
                              const int32_t* indices);
/* Model upload (InitModel is host-side RNG work: MatrixFactorization.cs:99-116). */
mml_status mml_bmf_set_model(mml_bmf* h, const float* user_factors, const float* item_factors,
                             const float* user_bias, const float* item_bias, float global_bias,
                             float min_rating, float max_rating);
mml_status mml_bmf_get_model(mml_bmf* h, float* user_factors, float* item_factors,
                             float* user_bias, float* item_bias);
/* InitModel on the device for models too large for the host RNG chain (C4: 640 M normals), after
 * set_data: N(mean, stddev) from a counter-based generator keyed by seed, rows of users / items
 * without training ratings 0 (MatrixFactorization.cs:99-116), biases 0.  Statistically, not
 * bitwise, equal to the MathNet draws; MML_MF_BIASED / MML_MF_PLAIN (ABI 4). */
mml_status mml_bmf_init_model(mml_bmf* h, uint64_t seed, double mean, double stddev,
                              float global_bias, float min_rating, float max_rating);
/* One epoch = BiasedMatrixFactorization.Iterate(IList<int>,bool,bool) (:264-310) -- for
 * MML_MF_PLAIN MatrixFactorization.Iterate(IList<int>,bool,bool) (MatrixFactorization.cs:166-196)
 * without its trailing UpdateLearnRate, which stays on the host -- over the stored
 * order at current_learnrate = learn_rate.  DSGD: subepoch_sequence[G] is the shuffled
 * sub-epoch order of Iterate() (:209-214); NULL otherwise. */
mml_status mml_bmf_iterate(mml_bmf* h, float learn_rate, const int32_t* subepoch_sequence);
/* BiasedMatrixFactorization.Predict(int,int) (:313-325), batched; unknown ids allowed.
 * MML_MF_PLAIN: MatrixFactorization.Predict(int,int) (MatrixFactorization.cs:251-258). */
mml_status mml_bmf_predict(mml_bmf* h, const int32_t* users, const int32_t* items, int64_t n,
                           float* out);
/* Eval.Ratings.Evaluate (Eval/Ratings.cs:96-139) on device: out[0] = RMSE, out[1] = MAE. */
mml_status mml_bmf_evaluate(mml_bmf* h, const int32_t* users, const int32_t* items,
                            const float* values, int64_t n, float* out);
/* Device time of the last mml_bmf_iterate's SGD kernels (HIP events on the library stream):
 * out[0] = ms for the whole epoch, out[1] = number of kernel launches in it. */
mml_status mml_bmf_last_timing(mml_bmf* h, float* out);
/* The dominant kernel of the last mml_bmf_iterate as rocprofv3 names the template instance, e.g.
 * "bmf_sgd_hogwild_kernel<0, 16, 1, 14>" or "bmf_sgd_ordered_kernel<0, 1>" (ABI 9; cleared by
 * every iterate, so empty after an epoch of the social / asymmetric models' kernels);
 * NUL-terminated, truncated to cap bytes. */
mml_status mml_bmf_last_kernel(mml_bmf* h, char* buf, int32_t cap);
/* BiasedMatrixFactorization.ComputeObjective (:496-552) on the device model and training data:
 * out[0] = ComputeLoss() (RMSE / MAE / logistic sum per params.loss, double), out[1] = the
 * complexity term; ComputeObjective = (float)(out[0] + out[1]).  BoldDriver's UpdateLearnRate
 * (:225-244) compares consecutive values on the host. */
mml_status mml_bmf_objective(mml_bmf* h, double* out);
/* The HOGWILD epoch's memory traffic without its arithmetic (ABI 10): the same launch over the same
 * stream, rows and biases with the same access flags, every loaded value stored back unchanged
 * (the model is not modified).  *out_ms = its device time: the access pattern's ceiling on the GPU
 * it runs on, which bench.py reports beside the epoch (frac_of_box_ceiling). */
mml_status mml_bmf_replay_traffic(mml_bmf* h, float* out_ms);
/* User phases of the HOGWILD epoch (ABI 10).  The XCD-partitioned stream is split into P phases by
 * a fixed hash of the user (the visit order kept within a phase) and the epoch runs one launch per
 * phase, so a launch touches 1/P of U and its rows stay in the 256 MB Infinity Cache between a
 * user's ratings.  phases = 0 (default): one phase per 96 MiB of the active users' rows, at most
 * 32 (C4: 26; C2: 3; sets under 96 MiB of U: 1); 1 = one launch over the whole stream.  Every
 * rating is still visited once per epoch.  mml_bmf_last_phases reports the count the last epoch
 * used. */
mml_status mml_bmf_set_hogwild_phases(mml_bmf* h, int32_t phases);
mml_status mml_bmf_last_phases(mml_bmf* h, int32_t* out);
/* User runs of the HOGWILD epoch (ABI 14).  Every XCD group's span is sorted by user (stably: a
 * user's ratings keep their visit order); the epoch runs as 8 launches over strata (users in 8
 * blocks of equal rating count; launch s gives group g block (g + s) mod 8, so no two XCDs hold one
 * user's row), and every lane group owns whole runs of one user: U_u and b_u are read once per run,
 * updated in registers rating after rating and written through once.  on = -1 (default): on from
 * 16 M ratings unless mml_bmf_set_hogwild_phases chose a phase count; 1: on; 0: off (the user
 * phases).  Needs U under 4 GiB and the XCD groups, else the phases run.  C4: ~110 ms per epoch
 * against 178-194 ms in 26 phases, the same RMSE.  The visit order changes:
 * mml_bmf_hogwild_stream exports it (launch-major, group-minor: 64 spans), and the sequential
 * Iterate() over it is the tests' reference (tests/test_runs_gpu.py).  mml_bmf_last_runs: the runs
 * of the last epoch (0: it ran without). */
mml_status mml_bmf_set_hogwild_runs(mml_bmf* h, int32_t on);
mml_status mml_bmf_last_runs(mml_bmf* h, int64_t* out);
/* The stream the last HOGWILD epoch ran on an 8-XCD device (ABI 13; single-device handles): the n
 * ratings (n = the handle's count) in the order the launches walk them -- phase-major, XCD-group
 * minor, the RandomIndex visit order kept inside a span -- and the phases * 8 + 1 span offsets
 * (phase p, group g = span p * 8 + g); *n_spans = phases * 8 (with user runs, ABI 14: the 8
 * launches' strata, launch s group g = span s * 8 + g, 64 spans).  The sequential Iterate()
 * (BiasedMatrixFactorization.cs:264-310) over this order is the epoch without Hogwild's concurrency
 * (tests/test_phases_c4_gpu.py).  MML_ERR_ARG before such an epoch. */
mml_status mml_bmf_hogwild_stream(mml_bmf* h, int32_t* users, int32_t* items, float* values,
                                  int64_t n, int64_t* span_offsets, int32_t cap_offsets,
                                  int32_t* n_spans);
/* Multi-GPU (user shards): in-place RCCL all-reduce of item factors and item
 * biases over the context's communicator with ncclAvg (model averaging).  Stream-ordered (ABI 6):
 * the call returns once the collective is enqueued; the next call on the handle runs after it. */
mml_status mml_bmf_allreduce_items(mml_bmf* h);
/* Device time of the last item average (ABI 6): mml_bmf_allreduce_items, or the average inside
 * a multi-device mml_bmf_iterate (RCCL: the slowest shard; peer copies: the whole average).
 * Waits for it to finish; 0 when none has run. */
mml_status mml_bmf_last_allreduce_ms(mml_bmf* h, float* out);
/* SocialMF.UserRelation (SocialMF.cs:50): rows [0, n_rows) of the user_connections
 * SparseBooleanMatrix as CSR (offsets[n_rows + 1], cols = the rows' HashSet enumeration order, no
 * duplicates within a row, ids < n_users); the library builds the Transpose() the batch step walks
 * (SparseBooleanMatrix.cs:200-207).  MML_MF_SOCIAL handles only. */
mml_status mml_bmf_set_user_relation(mml_bmf* h, int32_t n_rows, const int64_t* offsets,
                                     const int32_t* cols);
/* IFoldInRatingPredictor.ScoreItems' FoldIn (RatingPrediction/IFoldInRatingPredictor.cs:42-48):
 * BiasedMatrixFactorization.FoldIn (:447-492) -- MML_MF_PLAIN: MatrixFactorization.FoldIn
 * (MatrixFactorization.cs:326-351) -- for n_fold new users at once against the trained item side,
 * one wavefront each.  User x's ratings are rated_items/rated_values[rated_off[x] ..
 * rated_off[x+1]) in visiting order (the host has shuffled them, Utils.Shuffle) and
 * init_factors[x * k ..] are its InitNormal draws (drawn before the shuffle).  num_iter = NumIter,
 * learn_rate = LearnRate, decay = Decay (MML_MF_PLAIN only; BiasedMatrixFactorization.FoldIn does
 * not decay).  out_vectors: [n_fold x (k + 1)] = (user bias, factors) for MML_MF_BIASED
 * (FOLD_IN_BIAS_INDEX = 0, :80-82), [n_fold x k] for MML_MF_PLAIN. */
mml_status mml_bmf_fold_in(mml_bmf* h, int32_t n_fold, const int64_t* rated_off,
                           const int32_t* rated_items, const float* rated_values,
                           const float* init_factors, int32_t num_iter, float learn_rate,
                           float decay, float* out_vectors);
/* RetrainUser / RetrainItem (ABI 8; MatrixFactorization.cs:142-160, BiasedMatrixFactorization.cs:
 * 419-431), the incremental-update hook behind AddRatings / UpdateRatings / RemoveRatings
 * (MatrixFactorization.cs:262-290, IncrementalRatingPredictor.cs:40-78).  For every listed
 * row r of side 0 (users) or 1 (items): its bias <- 0 (MML_MF_BIASED), its factors <-
 * init_factors[x * k ..] (the row's RowInitNormal draws, DataType/MatrixExtensions.cs:35-42, drawn
 * by the caller in list order), then num_iter x Iterate(ByUser[r] / ByItem[r], side == 0,
 * side == 1) (:264-310; MatrixFactorization.cs:166-196): rated_ids[rated_off[x] .. rated_off[x+1])
 * are the other side's ids of the row's ratings in rating-index order, rated_values their values,
 * learn_rates[x * num_iter + it] the current_learnrate of that Iterate call (MatrixFactorization's
 * decays per call, BiasedMatrixFactorization's does not; the caller carries it).  The other side
 * stays fixed, so the rows are independent and run at once with the ORDERED kernel's exact
 * arithmetic; a row may be listed once.  MML_MF_BIASED and MML_MF_PLAIN, single-device handles. */
mml_status mml_bmf_retrain(mml_bmf* h, int32_t side, int32_t n_rows, const int32_t* rows,
                           const int64_t* rated_off, const int32_t* rated_ids,
                           const float* rated_values, const float* init_factors,
                           int32_t num_iter, const float* learn_rates);
/* Predict(float[] user_vector, int item_id) (BiasedMatrixFactorization.cs:327-335; MML_MF_PLAIN:
 * MatrixFactorization.cs:222-241, bound) for n (vector, item) pairs: vectors as mml_bmf_fold_in
 * writes them, vector_index[x] selects the vector of pair x.  MML_MF_PLAIN rejects items beyond the
 * model (the reference's RowScalarProduct throws). */
mml_status mml_bmf_predict_vectors(mml_bmf* h, int32_t n_vectors, const float* vectors,
                                   const int32_t* vector_index, const int32_t* items, int64_t n,
                                   float* out);

/* The asymmetric models' implicit feedback (ABI 3), one call per side the model uses.
 * side 0 (MML_MF_ITEM_ASYM, MML_MF_COMBINED_ASYM): lists = the items_rated_by_user CSR
 *   (ITransductiveRatingPredictor.ItemsRatedByUser, ITransductiveRatingPredictor.cs:63-79: per
 *   user the training items in rating-index order, then AdditionalFeedback's, distinct;
 *   n_rows = n_users), factors = y [n_items x k] (e.g. SigmoidItemAsymmetricFactorModel.cs:
 *   290-301), reg = y_reg [n_items] (Train :72-77).  U then holds PrecomputeUserFactors.
 * side 1 (MML_MF_USER_ASYM, MML_MF_COMBINED_ASYM): lists = UsersWhoRated (:40-55;
 *   n_rows = n_items), factors = x [n_users x k], reg = x_reg [n_users].  V then holds
 *   PrecomputeItemFactors.
 * The precomputed factors are refreshed after every epoch, so Predict / evaluate read the
 * reference's user_factors / item_factors. */
mml_status mml_bmf_set_implicit_feedback(mml_bmf* h, int32_t side, int32_t n_rows,
                                         const int64_t* offsets, const int32_t* ids,
                                         const float* factors, const float* reg);
/* y [n_items x k] (side 0) / x [n_users x k] (side 1), e.g. for SaveModel */
mml_status mml_bmf_get_implicit_factors(mml_bmf* h, int32_t side, float* factors);
/* SVD++: the free user factors p [n_users x k] (SVDPlusPlus.InitModel, SVDPlusPlus.cs:129-155);
 * together with side 0 they form the precomputed user factors (PrecomputeFactors :230-246) */
mml_status mml_bmf_set_user_offsets(mml_bmf* h, const float* p);
mml_status mml_bmf_get_user_offsets(mml_bmf* h, float* p);

/* ------------------------------------------------------------------ BPRMF */
enum {
    MML_BPR_SAMPLER_UNIFORM_USER = 0, /* default: IterateWithoutReplacementUniformUser (BPRMF.cs:216-226) */
    MML_BPR_SAMPLER_UNIFORM_PAIR = 1, /* IterateWithoutReplacementUniformPair over the visit order
                                         (:248-268; MultiCoreBPRMF's sampler, MultiCoreBPRMF.cs:49-63) */
    MML_BPR_SAMPLER_WEIGHTED = 2,     /* WeightedBPRMF.SampleTriple (WeightedBPRMF.cs:55-67): (u, i) a
                                         uniform event, j the item of a uniform event, not in S_u */
    MML_BPR_SAMPLER_USER_REPLACEMENT = 3, /* IterateWithReplacementUniformUser (BPRMF.cs:183-211):
                                         u uniform; i drawn WITHOUT repetition from the user's
                                         remaining items of this epoch, the set refilled when
                                         exhausted; j uniform outside S_u (ABI 3) */
    MML_BPR_SAMPLER_PAIR_REPLACEMENT = 4  /* IterateWithReplacementUniformPair (:231-243): (u, i) the
                                         event at a uniform index, j = SampleOtherItem (ABI 3) */
};
/* How an epoch's sampled triples are applied (ABI 2) */
enum {
    MML_BPR_SCHEDULE_AUTO = 0,    /* ORDERED for epochs under 262,144 samples, else HOGWILD */
    MML_BPR_SCHEDULE_HOGWILD = 1, /* lock-free: thousands of wavefronts, LPR lanes per triple */
    MML_BPR_SCHEDULE_ORDERED = 2  /* one wavefront applies the triples in sample order, exactly as
                                     the reference's loop (mml_bpr_apply_triples' kernel) */
};
/* UpdateFactors of the model family (ABI 2) */
enum {
    MML_BPR_MODEL_BPR = 0,        /* BPRMF.UpdateFactors (BPRMF.cs:330-374) */
    MML_BPR_MODEL_SOFT_MARGIN = 1 /* SoftMarginRankingMF.UpdateFactors (SoftMarginRankingMF.cs:66-113):
                                     hinge loss, no update when x_uij > 0 */
};

typedef struct {
    int32_t num_factors; /* NumFactors (MF.cs:43-45) */
    int32_t sampler;     /* MML_BPR_SAMPLER_*: UniformUserSampling / WithReplacement (BPRMF.cs:79-82) */
    int32_t update_j;    /* UpdateJ (:100) */
    float learn_rate;    /* LearnRate (:88) */
    float reg_u;         /* RegU (:91) */
    float reg_i;         /* RegI (:94) */
    float reg_j;         /* RegJ (:97) */
    float bias_reg;      /* BiasReg (:85) */
    int32_t model;       /* MML_BPR_MODEL_* (ABI 2) */
    int32_t schedule;    /* MML_BPR_SCHEDULE_* (ABI 2) */
} mml_bpr_params;

typedef struct mml_bpr mml_bpr;

mml_status mml_bpr_create(mml_ctx* ctx, const mml_bpr_params* params, int32_t n_users,
                          int32_t n_items, mml_bpr** out);
mml_status mml_bpr_destroy(mml_bpr* h);
/* Positive-only events (PosOnlyFeedback, Data/PosOnlyFeedback.cs:32-206; duplicates allowed and
 * counted in Feedback.Count = samples per epoch); order = Feedback.RandomIndex for UNIFORM_PAIR. */
mml_status mml_bpr_set_data(mml_bpr* h, const int32_t* users, const int32_t* items, int64_t n,
                            const int32_t* order);
/* Same from arrays already in this context's HBM; the sets are built on the device (csr.hip).
 * On a multi-device context (ABI 9) the arrays live on the first listed device, which splits them
 * into the user shards (as mml_bpr_set_data) and hands each device its part. */
mml_status mml_bpr_set_data_device(mml_bpr* h, const int32_t* users_device,
                                   const int32_t* items_device, int64_t n,
                                   const int32_t* order_device);
/* Model upload / download: U [n_users x k], V [n_items x k], item_bias [n_items]
 * (InitModel: MF.cs:51-58 + BPRMF.cs:121-126). */
mml_status mml_bpr_set_model(mml_bpr* h, const float* user_factors, const float* item_factors,
                             const float* item_bias);
mml_status mml_bpr_get_model(mml_bpr* h, float* user_factors, float* item_factors,
                             float* item_bias);
/* InitModel on the device for models too large for the host RNG chain (C3: 1.4e9 normals):
 * N(mean, stddev) from a counter-based generator keyed by seed; item biases = 0.  Statistically,
 * not bitwise, equal to MF.InitModel's MathNet draws (MF.cs:51-58). */
mml_status mml_bpr_init_model(mml_bpr* h, uint64_t seed, double mean, double stddev);
/* One epoch = BPRMF.Iterate() (:160-178): Feedback.Count sampled triples, each followed by
 * UpdateFactors (:330-374).  seed keys the counter-based sampler (e.g. drawn from the host RNG). */
mml_status mml_bpr_iterate(mml_bpr* h, uint64_t seed);
/* The seed the NEXT mml_bpr_iterate will be called with (ABI 12).  The following mml_bpr_iterate
 * then draws that epoch's triples on a second stream beside its own update (the triples depend on
 * the seed and the data only, not on the model), and the epoch after it starts at its update.
 * The same triples either way: an iterate with another seed draws its own.  One-shot; applies to
 * the partitioned HOGWILD epoch without user phases (not WEIGHTED, not USER_REPLACEMENT); costs a
 * second set of triple buffers (28 bytes per event).  A multi-device handle passes seed + d x
 * 0x9E3779B97F4A7C15 to device d, as mml_bpr_iterate does. */
mml_status mml_bpr_set_next_seed(mml_bpr* h, uint64_t seed);
/* UpdateFactors(u[x], i[x], j[x], true, true, UpdateJ) for x = 0 .. n-1 strictly in order, with
 * the reference's arithmetic and summation order (bit-faithful to the managed loop): the exact
 * path for a host that draws its own triples (e.g. the C# SampleTriple on System.Random). */
mml_status mml_bpr_apply_triples(mml_bpr* h, const int32_t* users, const int32_t* items,
                                 const int32_t* other_items, int64_t n);
/* The same with UpdateFactors' update_u / update_i / update_j per triple (ABI 8; flags[x] bits 0,
 * 1, 2; BPRMF.cs:330-374): RetrainUser (:391-402) applies its SampleItemPair triples with u only,
 * RetrainItem (:405-422) its SampleUser / SampleOtherItem triples with the retrained item only,
 * strictly in order on one wavefront. */
mml_status mml_bpr_apply_triples_flags(mml_bpr* h, const int32_t* users, const int32_t* items,
                                       const int32_t* other_items, const uint8_t* flags,
                                       int64_t n);
/* Overwrite factor rows (ABI 8): side 0 user rows, 1 item rows, values [n_rows x num_factors]
 * row-major, in list order (RowInitNormal of RetrainUser / RetrainItem, DataType/
 * MatrixExtensions.cs:35-42, drawn on the host); biases untouched. */
mml_status mml_bpr_set_rows(mml_bpr* h, int32_t side, int32_t n_rows, const int32_t* rows,
                            const float* values);
/* BPRMF.Predict (:425-431), batched: float.MinValue for ids beyond the model. */
mml_status mml_bpr_predict(mml_bpr* h, const int32_t* users, const int32_t* items, int64_t n,
                           float* out);
/* out[0] = the last epoch's device time (ms), out[1] = its update kernel alone (the rest is the
 * triple sampler; with mml_bpr_set_next_seed, the part of the next epoch's sampling that the
 * update did not cover) */
mml_status mml_bpr_last_timing(mml_bpr* h, float* out);
/* Device time of the last item average (ABI 10): mml_bpr_allreduce_items on a communicator, or the
 * peer-copy average inside a repeated-device mml_bpr_iterate; waits for it; 0 when none ran. */
mml_status mml_bpr_last_allreduce_ms(mml_bpr* h, float* out);
/* The last HOGWILD epoch's update launch again without its arithmetic (ABI 10): the same triples,
 * rows, biases, geometry and access flags, every loaded value stored back unchanged (the model is
 * not modified).  *out_ms = its device time, the access pattern's ceiling on this GPU (bench.py
 * frac_of_box_ceiling).  Needs a BPRMF (not SoftMargin) HOGWILD epoch before it. */
mml_status mml_bpr_replay_traffic(mml_bpr* h, float* out_ms);
/* The update kernel of the last Hogwild epoch as rocprofv3 names it, e.g.
 * "bpr_update_kernel<32, false, 27>" (ABI 9); NUL-terminated, truncated to cap bytes. */
mml_status mml_bpr_last_kernel(mml_bpr* h, char* buf, int32_t cap);
/* The HOGWILD epoch's launch width (ABI 10): 0 = the default (at least 65,536 triples per wave,
 * at most 8,192 waves: C3's 500 M events run 7,648); waves > 0 = that many waves, at least 32,
 * rounded up to a multiple of 32 (8 XCD groups x 4 waves), at most 8,192.  Lets a smaller set replay a larger
 * set's triples in flight -- the Hogwild staleness -- e.g. the C3-density AUC parity test.  No
 * effect on the ORDERED schedule or on epochs below 16 waves' worth of triples. */
mml_status mml_bpr_set_hogwild_waves(mml_bpr* h, int64_t waves);
/* User phases of the default sampler's HOGWILD epoch (ABI 10; the BiasedMF form is
 * mml_bmf_set_hogwild_phases).  The eligible users are split into P phases by a fixed hash; the
 * sampler draws the epoch's triples phase by phase -- each phase's share of the Feedback.Count
 * triples in proportion to its users, u uniform within the phase, so every user keeps SampleUser's
 * probability 1 / n_eligible per triple (BPRMF.cs:300-310) -- and each phase is partitioned by
 * XCD group and updated by its own launch, which then touches 1/P of U.  phases = 0 (default) or
 * 1: one draw over all users -- at C3 the phases were measured slower (update kernel 300 ms in one
 * phase, 304-313 ms in 32-64: the uniform V_j rows stream through the Infinity Cache between a
 * user's triples); P in [2, 64] turns them on.  mml_bpr_last_phases: the count the last epoch used. */
mml_status mml_bpr_set_hogwild_phases(mml_bpr* h, int32_t phases);
mml_status mml_bpr_last_phases(mml_bpr* h, int32_t* out);
/* The last epoch's sampled triples in sample order (n = Feedback.Count), e.g. for BPRMF's
 * loss_sample_* arrays (BPRMF.cs:136-150) or to check a sampler's distribution (ABI 3).  On a
 * multi-device context: each user shard's triples in its sample order, shard after shard (ABI 9;
 * shard d holds the events of its user range, mml_bpr_set_data's equal-count bounds). */
mml_status mml_bpr_last_triples(mml_bpr* h, int32_t* users, int32_t* items, int32_t* other_items,
                                int64_t n);
/* Eval.Items.Evaluate's AUC (Eval/Items.cs:126-209 + Recommender.Recommend n = -1 +
 * Eval/Measures/AUC.cs:42-68) on the device for the eval users: candidates = the already shuffled
 * candidate list (Items.Candidates, :62-96), the users' test items as CSR (test_off[n_users + 1],
 * distinct items per user); the training items of the handle's data are ignored per user.
 * out_auc[x] = that user's AUC, NaN for users the reference skips (no relevant candidate, or
 * only relevant ones).  The host averages (float accumulation, Items.cs:177-188). */
mml_status mml_bpr_auc(mml_bpr* h, const int32_t* candidates, int32_t n_candidates,
                       const int32_t* users, int32_t n_users, const int64_t* test_off,
                       const int32_t* test_items, double* out_auc);
/* Multi-GPU (user shards): RCCL all-reduce of item factors + item biases with ncclAvg (model
 * averaging), stream-ordered like mml_bmf_allreduce_items (ABI 6).  The WEIGHTED sampler is
 * single-device only (its j draws follow the global item popularity). */
mml_status mml_bpr_allreduce_items(mml_bpr* h);

/* ------------------------------------------------------------------ WRMF */
typedef struct {
    int32_t num_factors;   /* NumFactors (MF.cs:43-45), <= 256: k <= 128 solves in fp64, k > 128
                              in fp32 on the matrix cores (A in fp64 does not fit the LDS) */
    int32_t refine_passes; /* k > 128 (ABI 5): at most this many passes of fp64 iterative
                              refinement after the fp32 solve, x += A^{-1} (b - A x) with the
                              residual in fp64 (exact float products); a further pass runs only
                              while the last correction exceeded 3e-4 relative on a direct row
                              or 2e-6 on a Woodbury row (the two solvers' contractions): one
                              pass reaches the fp64 solution on well-conditioned systems,
                              cond ~1e4 takes two (WRMF.cs:137-154); 0 = the fp32 result */
    double alpha;          /* Alpha (WRMF.cs:56) */
    double regularization; /* Regularization (WRMF.cs:59) */
} mml_wrmf_params;

typedef struct mml_wrmf mml_wrmf;

mml_status mml_wrmf_create(mml_ctx* ctx, const mml_wrmf_params* params, int32_t n_users,
                           int32_t n_items, mml_wrmf** out);
mml_status mml_wrmf_destroy(mml_wrmf* h);
/* Positive-only events; the user->items and item->users sets (Feedback.UserMatrix / ItemMatrix,
 * Data/PosOnlyFeedback.cs:35-83) are built from them. */
mml_status mml_wrmf_set_data(mml_wrmf* h, const int32_t* users, const int32_t* items, int64_t n);
mml_status mml_wrmf_set_data_device(mml_wrmf* h, const int32_t* users_device,
                                    const int32_t* items_device, int64_t n);
/* InitModel on the device (counter-based N(mean, stddev)); see mml_bpr_init_model. */
mml_status mml_wrmf_init_model(mml_wrmf* h, uint64_t seed, double mean, double stddev);
mml_status mml_wrmf_set_model(mml_wrmf* h, const float* user_factors, const float* item_factors);
mml_status mml_wrmf_get_model(mml_wrmf* h, float* user_factors, float* item_factors);
/* One WRMF.Iterate() (WRMF.cs:68-73): Optimize(users | items) then Optimize(items | users),
 * each = ComputeSquareMatrix (:94-108) + one k x k solve per row (:110-156), fp64. */
mml_status mml_wrmf_iterate(mml_wrmf* h);
/* WRMF.RetrainUser / RetrainItem (ABI 8; ItemRecommendation/WRMF.cs:159-170), the hook behind
 * MF.AddFeedback / RemoveFeedback (ItemRecommendation/MF.cs:73-99): for every listed row r of
 * side 0 (users) or 1 (items), Optimize(r) against the fixed other side with HH recomputed from it
 * (ComputeSquareMatrix).  rated_ids[rated_off[x] .. rated_off[x+1]) are the other side's ids of
 * row x's feedback (Feedback.UserMatrix / ItemMatrix row).  The rows are independent, so they run
 * as one half-step over their own CSR with the iterate's solvers and precision; a row may be
 * listed once.  Single-device handles. */
mml_status mml_wrmf_retrain(mml_wrmf* h, int32_t side, int32_t n_rows, const int32_t* rows,
                            const int64_t* rated_off, const int32_t* rated_ids);
/* MF.Predict (MF.cs:151-157): float.MinValue for ids beyond the model. */
mml_status mml_wrmf_predict(mml_wrmf* h, const int32_t* users, const int32_t* items, int64_t n,
                            float* out);
mml_status mml_wrmf_last_timing(mml_wrmf* h, float* out);
/* Device time of the last mml_wrmf_iterate's two row-shard all-gathers (ABI 10; U after the user
 * half, V after the item half; the slowest shard on a multi-device context); 0 on one rank. */
mml_status mml_wrmf_last_allgather_ms(mml_wrmf* h, float* out);
/* The item half's pipeline (ABI 11; 128 < k <= 256, fp64 mode): the direct rows of a half-step with
 * no Woodbury rows are solved in `ranges` contiguous row ranges, and range b's first refinement
 * residual runs on a second stream under range b + 1's solve; HH of such a half is computed on that
 * stream under the hot rows' split Gram.  The model is the serial path's bit for bit.  ranges = 0
 * (default): 12 ranges, or one per 4,096 direct rows where a half has fewer, and none below
 * 4 x 4,096 direct rows (round 5's default was 4 ranges); 1: off; 2 .. 16: that many where the half
 * has >= 4,096 direct rows per range.  Takes effect at the next mml_wrmf_iterate. */
mml_status mml_wrmf_set_pipeline(mml_wrmf* h, int32_t ranges);
/* The most refinement passes a half-step of the last mml_wrmf_iterate ran (ABI 6);
 * corrections (nullable, [8]): per half-step (users 0..3, items 4..7) and pass, the largest
 * correction relative to 1 + |x| that decided whether another pass ran (0: not read back). */
mml_status mml_wrmf_last_refine_passes(mml_wrmf* h, int32_t* out, float* corrections);
/* As mml_bpr_auc for the WRMF (MF.Predict) scorer. */
mml_status mml_wrmf_auc(mml_wrmf* h, const int32_t* candidates, int32_t n_candidates,
                        const int32_t* users, int32_t n_users, const int64_t* test_off,
                        const int32_t* test_items, double* out_auc);

#ifdef __cplusplus
}
#endif

#endif /* MML_H */
