/*
 * pgm_abi.h -- C ABI of libpgm.so, the MI355X (gfx950) kernels of the PG-MORL MOPG hot path.
 *
 * Every entry point is batched over P tasks (policies), takes CALLER-OWNED device buffers
 * (plain pointers; no allocation inside), is ordered on the passed hipStream_t and returns
 * an int status (PGM_OK or a negative PGM_E_*).  pgm_last_error() returns a thread-local
 * message for the last failure.  No global mutable state besides that string, the pre-zeroed-workspace
 * marks of pgm_ppo_update_reset (mutex-guarded) and a per-device CU count (an immutable device property):
 * no cached launch decisions, no allocation inside the library, and no environment variables read: every
 * launch choice is an argument (pgm_launch_opts).  Calls on distinct streams are independent.  One host
 * thread per device.
 *
 * Reference seams replaced (albo437/PGMORL; paths relative to the reference tree):
 *   pgm_act_forward       Policy.act / get_value            a2c_ppo_acktr/model.py:57-73
 *                          (+ DiagGaussian sample/log_prob   a2c_ppo_acktr/distributions.py:29-40,71-90)
 *   pgm_env_reset         envs.reset() through VecNormalize  baselines/.../vec_env/vec_normalize.py:63-66
 *   pgm_env_step          envs.step(): DummyVecEnv auto-reset + TimeLimitMask + VecNormalize
 *                          + VecPyTorch fp32 cast + mask/bad_mask bookkeeping
 *                                                           dummy_vec_env.py:45-56, a2c_ppo_acktr/envs.py:122-131,
 *                                                           171-217, vec_normalize.py:29-61, morl/mopg.py:110-130
 *   pgm_rollout           the T-step rollout loop + bootstrap value (morl/mopg.py:103-135 with
 *                          RolloutStorage.insert a2c_ppo_acktr/storage.py:50-62)
 *   pgm_gae               RolloutStorage.compute_returns    a2c_ppo_acktr/storage.py:77-116
 *   pgm_adv_normalize     PPO.update advantage prologue     a2c_ppo_acktr/algo/ppo.py:41-56
 *                          + WeightedSumScalarization        morl/scalarization_methods.py:28-29
 *   pgm_ppo_update        PPO.update epochs x minibatches   a2c_ppo_acktr/algo/ppo.py:58-115
 *                          (+ feed_forward_generator storage.py:118-154, clip_grad_norm_, Adam)
 *                          (pgm_ppo_update_reset: its workspace reset, issued ahead on another stream)
 *   pgm_eval              evaluation()                       morl/mopg.py:25-46
 *   pgm_randperm          SubsetRandomSampler's randperm     (perf-mode RNG replacement)
 *   pgm_normal_noise      Normal.sample's torch.normal draw  (perf-mode RNG replacement)
 *
 * Layouts (row-major, fp32 unless noted; P = tasks, N = envs per task, T = rollout steps,
 * O/A/K = obs/action/objective dims, H = hidden width, fixed 64 in this build):
 *   params/adam_m/adam_v  [P][L]  L and tensor offsets from pgm_param_layout (weights stored
 *                                 TRANSPOSED, [in][out]; see DESIGN.md "Data layout in HBM")
 *   rollout buffers       obs [P][T+1][N][O], actions [P][T][N][A], logp [P][T][N],
 *                         values/returns [P][T+1][N][K], rewards [P][T][N][K],
 *                         masks/bad_masks [P][T+1][N], adv [P][T][N]
 *   env state (fp64)      s [P][N][O], elapsed int32 [P][N], obj_acc [P][N][K], obj_acc_valid int32 [P],
 *                         ret [P][N]
 *   running stats (fp64)  ob_mean/var [P][O], ob_count [P], ret_* [P], obj_mean/var [P][K], obj_count [P]
 *   shared RNG inputs     noise [T][N][A] fp32 and perms [E][T*N] int32 are shared by all tasks, as in the
 *                         reference where every task process reseeds torch with the iteration index
 *                         (morl/mopg.py:96).
 */
#ifndef PGM_ABI_H
#define PGM_ABI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PGM_ABI_VERSION 4

#define PGM_OK 0
#define PGM_E_INVALID_ARG (-1)
#define PGM_E_SHAPE (-2)
#define PGM_E_HIP (-3)
#define PGM_E_UNSUPPORTED (-4)

/* Parameter tensors in reference named_parameters() order (model.py:201-256, distributions.py:71-79). */
#define PGM_P_ACTOR_W1 0   /* base.actor.0.weight^T   [O][H] */
#define PGM_P_ACTOR_B1 1   /* base.actor.0.bias       [H]    */
#define PGM_P_ACTOR_W2 2   /* base.actor.2.weight^T   [H][H] */
#define PGM_P_ACTOR_B2 3   /* base.actor.2.bias       [H]    */
#define PGM_P_CRITIC_W1 4  /* base.critic.0.weight^T  [O][H] */
#define PGM_P_CRITIC_B1 5
#define PGM_P_CRITIC_W2 6  /* base.critic.2.weight^T  [H][H] */
#define PGM_P_CRITIC_B2 7
#define PGM_P_VALUE_W 8    /* base.critic_linear.weight^T [H][K] */
#define PGM_P_VALUE_B 9    /* base.critic_linear.bias [K] */
#define PGM_P_MEAN_W 10    /* dist.fc_mean.weight^T   [H][A] */
#define PGM_P_MEAN_B 11    /* dist.fc_mean.bias       [A] */
#define PGM_P_LOGSTD 12    /* dist.logstd._bias       [A] (reference shape [A][1]) */
#define PGM_NUM_PARAM_TENSORS 13

typedef void* pgm_stream_t; /* a hipStream_t (0 = the null stream) */

typedef struct pgm_dims {
    int32_t P, N, T, O, A, K, H;
} pgm_dims;

typedef struct pgm_env_spec { /* device pointers, fp64 */
    const double* d;      /* [O]    */
    const double* U;      /* [O][A] */
    const double* c;      /* [O]    */
    const double* V;      /* [K][O] */
    const double* ebase;  /* [K]    */
    const double* ecoef;  /* [K]    */
    const double* act_lo; /* [A]    */
    const double* act_hi; /* [A]    */
    int32_t max_episode_steps;
    int32_t _pad;
} pgm_env_spec;

typedef struct pgm_env_state { /* device pointers */
    double* s;              /* [P][N][O] */
    int32_t* elapsed;       /* [P][N]    */
    double* obj_acc;        /* [P][N][K] */
    int32_t* obj_acc_valid; /* [P]       */
    double* ret;            /* [P][N]    */
    const double* s0;       /* [N][O] reset state of env rank n (seed + n) */
} pgm_env_state;

typedef struct pgm_norm_state { /* device pointers (fp64) + flags */
    double *ob_mean, *ob_var, *ob_count;
    double *ret_mean, *ret_var, *ret_count;
    double *obj_mean, *obj_var, *obj_count;
    double gamma, clipob, cliprew, epsilon;
    int32_t use_ob_rms, use_obj_rms;
} pgm_norm_state;

typedef struct pgm_rollout_buf { /* device pointers */
    float* obs;
    float* actions;
    float* logp;
    float* values;
    float* rewards;
    float* masks;
    float* bad_masks;
    float* returns;
    float* adv;
} pgm_rollout_buf;

/* Launch options (ABI 4; no reference counterpart): which kernel family pgm_rollout / pgm_eval / pgm_ppo_update may
 * launch.  All zero, or a NULL pointer, = the automatic rule documented at each entry point.  The library reads no
 * environment variables; pgmorl_amd/_lib.py maps PGM_UPDATE_KERNEL / PGM_UPDATE_SPLIT / PGM_FS_DUAL /
 * PGM_ROLLOUT_KERNEL / PGM_EVAL_KERNEL onto this struct (A/B runs and tests). */
#define PGM_UPDATE_AUTO 0     /* feature-split while it gets >= 4 parts per tower, else the row split */
#define PGM_UPDATE_FS 1       /* the feature-split update wherever it fits */
#define PGM_UPDATE_ROWSPLIT 2 /* the row-split MFMA kernels (t16, MODE 2 / 1 / 0) */
#define PGM_UPDATE_VALU 3     /* the VALU reference update (obs_dim <= 64; A/B only) */
#define PGM_SPLIT_AUTO 0      /* row split: as many workgroups per tower as fit the device */
#define PGM_SPLIT_TASK 1      /* at most one workgroup per task (MODE 0; wide: one per tower) */
#define PGM_SPLIT_TOWER 2     /* at most one workgroup per tower (MODE 1; wide NS 1) */
#define PGM_SPLIT_HALVES 3    /* at most two per tower (MODE 2; wide NS 2) */
#define PGM_SPLIT_QUARTERS 4  /* at most four per tower (t16; wide NS 4) */
typedef struct pgm_launch_opts {
    int32_t update_kernel;   /* PGM_UPDATE_*; obs_dim <= 32 with update_split != AUTO means ROWSPLIT */
    int32_t update_split;    /* PGM_SPLIT_* (row-split and wide updates) */
    int32_t fs_one_per_cu;   /* 1: the feature-split update never places two workgroups on one CU */
    int32_t rollout_kernel;  /* 0 automatic (lane / wide kernels), 1 the workgroup-per-step kernel (A/B, tests) */
    int32_t eval_kernel;     /* 0 automatic (wave / wide kernels), 1 the workgroup-per-step kernel (A/B, tests) */
    int32_t _pad;
} pgm_launch_opts;

typedef struct pgm_ppo_hparams {
    float clip_param, value_loss_coef, entropy_coef, max_grad_norm;
    float adam_eps, beta1, beta2, _pad;
    int32_t ppo_epoch, num_mini_batch, use_clipped_value_loss, _pad2;
} pgm_ppo_hparams;

int pgm_abi_version(void);
const char* pgm_last_error(void);

/* Flat per-task parameter layout: offsets[PGM_NUM_PARAM_TENSORS] (floats) and the padded
 * per-task length *total (a multiple of 64 floats). */
int pgm_param_layout(int32_t O, int32_t A, int32_t K, int32_t H, int32_t* offsets, int32_t* total);

/* Policy.act on obs [P][N][O] (model.py:57-69).  noise [N][A] (shared by tasks) gives
 * action = noise*exp(logstd) + mean; deterministic=1 gives action = mean (noise ignored).
 * Outputs value [P][N][K], action [P][N][A], logp [P][N]. */
int pgm_act_forward(const pgm_dims* d, const float* params, const float* obs, const float* noise,
                    int32_t deterministic, float* value, float* action, float* logp, pgm_stream_t stream);

/* envs.reset(): every env to its reset state, VecNormalize.ret = 0, ob_rms update + normalise.
 * Also clears elapsed and VecNormalize.obj (a fresh make_vec_envs, morl/mopg.py:67-81).
 * Writes obs_out [P][N][O]. */
int pgm_env_reset(const pgm_dims* d, const pgm_env_spec* spec, const pgm_env_state* st,
                  const pgm_norm_state* ns, float* obs_out, pgm_stream_t stream);

/* One envs.step(action [P][N][A]) -> obs_out [P][N][O], reward_out [P][N][K] (info['obj'] after
 * obj_rms scaling), masks_out/bad_masks_out [P][N]. */
int pgm_env_step(const pgm_dims* d, const pgm_env_spec* spec, const pgm_env_state* st,
                 const pgm_norm_state* ns, const float* action, float* obs_out, float* reward_out,
                 float* masks_out, float* bad_masks_out, pgm_stream_t stream);

/* The fused rollout: for t in [0,T): act on obs[t] -> env step -> insert (storage.py:50-62),
 * then values[T] = get_value(obs[T]).  carry=1 first applies after_update() (obs/masks/bad_masks
 * slot T -> 0, storage.py:71-75).  noise [T][N][A] or NULL: NULL draws the perf-mode counter RNG of
 * pgm_normal_noise keyed by seed (the iteration index). */
int pgm_rollout(const pgm_dims* d, const float* params, const pgm_env_spec* spec, const pgm_env_state* st,
                const pgm_norm_state* ns, const pgm_rollout_buf* rb, const float* noise, uint64_t seed,
                int32_t carry, const pgm_launch_opts* opts, pgm_stream_t stream);

/* compute_returns(next_value already in values[T], use_gae, gamma, lam, use_proper_time_limits). */
int pgm_gae(const pgm_dims* d, const pgm_rollout_buf* rb, float gamma, float lam, int32_t use_gae,
            int32_t use_proper_time_limits, pgm_stream_t stream);

/* adv [P][T][N] = normalise(w . (R * s) - w . (V * s)), s = sqrt(obj_var + 1e-8) (or 1 if obj_var
 * is NULL); mean and UNBIASED std over T*N, (x - mean) / (std + 1e-5).  weights/obj_var [P][K] fp64. */
int pgm_adv_normalize(const pgm_dims* d, const pgm_rollout_buf* rb, const double* weights,
                      const double* obj_var, pgm_stream_t stream);

/* PPO.update minibatch loop: ppo_epoch x (T*N / (T*N/num_mini_batch)) Adam steps per task, rows
 * perms[e][b*mb:(b+1)*mb].  params/adam_m/adam_v [P][L] updated in place, adam_step [P] int32
 * incremented per step, lr [P].  stats [P][3] = mean (value_loss, action_loss, dist_entropy).
 * workspace: caller-owned device bytes (pgm_ppo_update_workspace_bytes), required (PGM_E_INVALID_ARG
 * when NULL), reset inside the call on `stream` unless pgm_ppo_update_reset did it since the last call.
 * The critic and actor towers of a task run on separate CUs that exchange the squared gradient norm per
 * minibatch step.  obs_dim <= 32 and small per-GPU populations (>= 4 parts per tower fit: 16 NS ceil(P/8) <= CUs,
 * or <= 2 x CUs with two workgroups per CU when each part takes two 16-row tiles; minibatch rows a multiple of 16 NS):
 * each tower on NS = 16 / 8 / 6 / 4 workgroups that split the minibatch rows, the four waves of a workgroup split the
 * hidden features, and the gradient is reduce-scattered over the parts before Adam (the feature-split update;
 * opts->fs_one_per_cu keeps one workgroup per CU).  Otherwise each tower is split over four CUs (a quarter of the minibatch rows each, gradient
 * images added through the workspace) while 64 * ceil(P/8) <= CU count, else over two CUs while
 * 32 * ceil(P/8) <= CU count (obs_dim > 32: 32 * ceil(P/4) / 16 * ceil(P/4)).  obs_dim <= 32: tower
 * images LDS-resident (falls back to 2 CUs per task, then 1, as P grows); obs_dim > 32 (Humanoid): layer
 * 1 streamed from L2, needs 2P <= CU count (PGM_E_UNSUPPORTED otherwise: shard the tasks over more
 * GPUs).  opts->update_split caps the row split; opts->update_kernel = PGM_UPDATE_FS forces the feature-split
 * update wherever it fits, PGM_UPDATE_ROWSPLIT the row-split kernels.
 * After the call, the 8-byte word at index 2P of the workspace is nonzero iff an exchange timed out
 * (the workgroups were not co-resident); the results of such a call are invalid. */
int pgm_ppo_update(const pgm_dims* d, const pgm_ppo_hparams* hp, float* params, float* adam_m,
                   float* adam_v, int32_t* adam_step, const float* lr, const int32_t* perms,
                   const pgm_rollout_buf* rb, float* stats, void* workspace, const pgm_launch_opts* opts,
                   pgm_stream_t stream);
/* Workspace bytes for dims d; monotone in d->P, so a workspace sized for P serves every call with P' <= P tasks
 * (the same other dims). */
size_t pgm_ppo_update_workspace_bytes(const pgm_dims* d);
/* The update kernel pgm_ppo_update would launch for these dims, hyper-parameters and opts on the current device
 * (the same selection rule), as text into buf[n]
 * (e.g. "ppo_update_fs_kernel (NS=16, R=1)", "... (NS=8, R=2, 2 per CU)"): what benchmarks and profiles report.  No reference
 * counterpart (diagnostic). */
int pgm_ppo_update_variant(const pgm_dims* d, const pgm_ppo_hparams* hp, const pgm_launch_opts* opts, char* buf,
                           int n);
/* Zero, on `stream`, the part of the workspace the next pgm_ppo_update for dims d would reset inside the call,
 * and let that call skip its own reset (the caller orders this stream before the update's stream and after
 * every read of the previous update's timeout word).  Lets a caller take the reset off the update's stream. */
int pgm_ppo_update_reset(const pgm_dims* d, void* workspace, pgm_stream_t stream);
/* The feature-split update's fragment map (diagnostic, no reference counterpart): for tower m (0 critic, 1 actor)
 * of dims (O, A, K), O <= 32, out[(b * 64 + l) * 4 + r] = the tower-image index the kernel keeps in register r of
 * lane l of exchange block b (-1: padding), for every block b < NB; returns NB or a negative status (cap = out's
 * length in entries, >= 256 NB).  Host-only, no device work. */
int pgm_ppo_fs_fragment_map(int32_t O, int32_t A, int32_t K, int32_t m, int32_t* out, int32_t cap);

/* evaluation(): eval_num deterministic episodes per task from s0_eval [eval_num][O], obs normalised
 * with the snapshot ob_mean/ob_var [P][O] (use_ob_rms), objs_out [P][K] fp64 (discounted by gamma
 * unless raw). */
int pgm_eval(const pgm_dims* d, const float* params, const pgm_env_spec* spec, const double* ob_mean,
             const double* ob_var, const double* s0_eval, int32_t eval_num, int32_t use_ob_rms, int32_t raw,
             double gamma, double* objs_out, const pgm_launch_opts* opts, pgm_stream_t stream);

/* count independent random permutations of [0, n) into out [count][n] (int32), keyed by seed. */
int pgm_randperm(int32_t n, int32_t count, uint64_t seed, int32_t* out, pgm_stream_t stream);

/* n standard-normal fp32 draws into out, element i keyed by (seed, i): the perf-mode noise stream. */
int pgm_normal_noise(int64_t n, uint64_t seed, float* out, pgm_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif
