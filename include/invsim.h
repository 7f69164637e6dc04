/* invsim — MI355X-native vectorised inventory-simulation engine: C ABI.
 *
 * This is the drop-in boundary for the reference's hot path, the Gymnasium
 * `Env.reset()` / `Env.step()` pair of the five environment classes of
 * jacklu2016/or-gym-inventory.  One handle = one batch of N independent env
 * instances of one class, resident in HBM (SoA state), bound to one GPU.
 *
 *   reference interface                                  replaced by
 *   ---------------------------------------------------  ----------------------------------
 *   NewsvendorEnv.__init__            newsvendor.py:52-97   invsim_create_newsvendor
 *   InvManagementMasterEnv.__init__   inventory_management.py:48-141
 *     (+ Backlog/LostSales subclasses :429-451)            invsim_create_invmgmt
 *   NetInvMgmtMasterEnv.__init__      network_management.py:55-106,146-195
 *     (+ Backlog/LostSales subclasses :747-770)            invsim_create_netinvmgmt
 *   gym.Env.reset(seed=s) -> seeding.np_random(s)
 *     (newsvendor.py:102, inventory_management.py:197,
 *      network_management.py:303)                          invsim_seed_range / invsim_seed_words
 *   Env.reset()  newsvendor.py:100-123,
 *                inventory_management.py:186-222,
 *                network_management.py:301-332              invsim_reset
 *   Env.step()   newsvendor.py:125-204,
 *                inventory_management.py:224-352,
 *                network_management.py:436-635              invsim_step
 *   K x Env.step() with pre-computed actions                invsim_rollout
 *   (no reference equivalent: env state is never
 *    checkpointed there)                                   invsim_state_* / invsim_get_state / invsim_set_state
 *
 * Conventions
 *  - Every buffer argument of reset/step/rollout/seed/state calls is a DEVICE
 *    pointer on the handle's GPU, owned by the caller.  Spec structs passed to
 *    invsim_create_* are HOST memory and are copied.
 *  - `stream` is a hipStream_t (NULL = default stream).  Calls are
 *    asynchronous on that stream; the library never synchronises.
 *  - Dtypes follow the reference spaces: Newsvendor obs/action f32;
 *    InvMgmt obs/action int64; NetInvMgmt obs/action f32.  Rewards f64.
 *    terminated/truncated are uint8 (0/1).
 *  - Return 0 on success, a negative errno-style code on failure;
 *    invsim_last_error(h) (or invsim_last_error(NULL) after a failed create)
 *    gives the message.  No exceptions cross the ABI.
 *  - A handle is not thread-safe.  One handle per GPU per process.
 */
#ifndef INVSIM_H
#define INVSIM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define INVSIM_ABI_VERSION 4   /* 2: market samplers appended to invsim_netinvmgmt_spec
                                  3: graph capture (invsim_capture_begin / _end, invsim_position)
                                  4: episode sink (invsim_set_episode_sink, invsim_episode_fold_groups) */

#define INVSIM_OK 0
#define INVSIM_EINVAL (-22)
#define INVSIM_ENOMEM (-12)
#define INVSIM_EDEVICE (-5)
#define INVSIM_ERANGE (-34)

/* Env families */
#define INVSIM_NEWSVENDOR 1
#define INVSIM_INVMGMT 2
#define INVSIM_NETINVMGMT 3

/* Vector autoreset modes (gymnasium.vector.AutoresetMode) */
#define INVSIM_AUTORESET_NEXT_STEP 0 /* gymnasium >= 1.0 default: reset on the step after done   */
#define INVSIM_AUTORESET_SAME_STEP 1 /* SB3 VecEnv: reset in the done step, final obs separately */
#define INVSIM_AUTORESET_DISABLED 2  /* caller resets explicitly                                   */

typedef struct invsim_handle invsim_handle;

/* newsvendor.py:52-61 constructor arguments */
typedef struct {
    int32_t lead_time;         /* <0 is clamped to 0 (:65); at most 128 */
    int32_t step_limit;
    double max_inventory;
    double max_order_quantity;
    double p_max, h_max, k_max, mu_max;
    double gamma;              /* accepted, unused by the dynamics (as in the reference) */
} invsim_newsvendor_spec;

/* inventory_management.py:48-101 after parameter processing.  Coefficient
 * arrays are the reference's float32 arrays (:89-92). */
typedef struct {
    int32_t num_stages;              /* m = len(I0) + 1, 2..9 */
    int32_t periods;
    int32_t backlog;                 /* 1 = InvManagementBacklogEnv, 0 = LostSales */
    int32_t dist;                    /* 1 Poisson(mu), 2 binomial(n, p), 3 integers(low, high + 1),
                                        4 geometric(p), 5 user_D  (inventory_management.py:169-184) */
    double mu;                       /* dist_param['mu'] */
    double alpha;                    /* discount; reward *= alpha**t */
    const int64_t *I0;               /* [m-1] */
    const float *unit_price;         /* [m] = append(p, r[:-1]) */
    const float *unit_cost;          /* [m] = r */
    const float *demand_cost;        /* [m] = k */
    const float *holding_cost;       /* [m] = append(h, 0) */
    const int64_t *supply_capacity;  /* [m-1] = c */
    const int64_t *lead_time;        /* [m-1] = L, each 0..255 */
    const int64_t *user_D;           /* [periods], dist == 5 only (else NULL) */
    int64_t dist_n;                  /* dist 2: dist_param['n'] */
    double dist_p;                   /* dist 2, 4: dist_param['p'] */
    int64_t dist_low, dist_high;     /* dist 3: dist_param['low'], ['high'] (inclusive) */
} invsim_invmgmt_spec;

/* network_management.py:146-195 classification, compiled to index tables by
 * the host (main nodes sorted; reorder links sorted; retail links in graph
 * edge order; adjacency lists in graph adjacency order). */
typedef struct {
    int32_t n_main;      /* J */
    int32_t n_reorder;   /* E  (= action dim) */
    int32_t n_retail;    /* RL */
    int32_t num_periods;
    int32_t backlog;     /* EFFECTIVE flag (the reference LostSales class runs backlog=True) */
    double alpha;
    /* main nodes [J] */
    const double *I0, *h, *C, *o, *v;
    const int32_t *is_factory, *is_retail;
    /* reorder links [E] */
    const int32_t *sup;             /* supplier main-node index, -1 = raw material */
    const int32_t *pur;             /* purchaser main-node index */
    const int32_t *sup_is_factory;
    const int32_t *L;               /* lead time, 0..255 */
    const double *lp, *lg;          /* price p, pipeline holding g */
    /* retail links [RL] */
    const int32_t *rl_node;         /* retailer main-node index */
    const double *rl_p, *rl_b, *rl_lam;
    const int32_t *rl_user;         /* 1: demand = user_D row (network_management.py:250-255) */
    const double *user_D;           /* [RL][num_periods] or NULL */
    /* CSR adjacency.  succ: successors of each main node (kind 0 = reorder link idx,
     * kind 1 = retail link idx); pred: reorder links into each main node. */
    const int32_t *succ_ptr;        /* [J+1] */
    const int32_t *succ_kind;       /* [succ_ptr[J]] */
    const int32_t *succ_idx;        /* [succ_ptr[J]] */
    const int32_t *pred_ptr;        /* [J+1] */
    const int32_t *pred_idx;        /* [pred_ptr[J]] */
    /* market demand samplers per retail link, the numpy Generator method the
     * edge's demand_dist_func calls with dist_param (network_management.py:
     * 125-127, 257-263; demand = max(0, int(round(draw)))).  rl_dist NULL = all
     * Poisson(rl_lam).  1 poisson(rl_lam), 2 binomial(rl_n, rl_dp),
     * 3 integers(rl_n, rl_high) (high exclusive), 4 geometric(rl_dp).  Graphs
     * with a non-Poisson market run the generic kernel. */
    const int32_t *rl_dist;
    const int64_t *rl_n, *rl_high;
    const double *rl_dp;
} invsim_netinvmgmt_spec;

int invsim_abi_version(void);
const char *invsim_last_error(const invsim_handle *h);

int invsim_create_newsvendor(const invsim_newsvendor_spec *spec, int64_t n_envs, int32_t device,
                             int32_t autoreset_mode, invsim_handle **out);
int invsim_create_invmgmt(const invsim_invmgmt_spec *spec, int64_t n_envs, int32_t device,
                          int32_t autoreset_mode, invsim_handle **out);
int invsim_create_netinvmgmt(const invsim_netinvmgmt_spec *spec, int64_t n_envs, int32_t device,
                             int32_t autoreset_mode, invsim_handle **out);
void invsim_destroy(invsim_handle *h);

/* obs_dim, action_dim, number of demand draws per step (info_demand width), env family */
int invsim_dims(const invsim_handle *h, int32_t *obs_dim, int32_t *action_dim, int32_t *demand_dim,
                int32_t *family);
int invsim_set_autoreset(invsim_handle *h, int32_t mode);

/* Seeding = gymnasium seeding.np_random(seed): numpy SeedSequence(seed) -> PCG64.
 * seed_range: env i (mask[i] != 0, or all when mask == NULL) gets the 128-bit
 * integer seed  base + first_index + i  (gymnasium SyncVectorEnv: seed + i).
 * seed_words: env i gets the little-endian uint32 entropy words[i][0..nwords[i]).
 * An unmasked seed (mask == NULL) also restarts the fast demand stream's
 * launch-step counter (INVSIM_DEMAND_PHILOX below), so reseeding every env with
 * the same seeds replays the same demands; a masked seed keeps the counter. */
int invsim_seed_range(invsim_handle *h, uint64_t base_lo, uint64_t base_hi, int64_t first_index,
                      const uint8_t *mask, void *stream);
int invsim_seed_words(invsim_handle *h, const uint32_t *words /*[N][4]*/,
                      const int32_t *nwords /*[N]*/, const uint8_t *mask, void *stream);

/* Env.reset() on every env (mask NULL) or on mask[i] != 0; writes obs rows of
 * the reset envs (obs may be NULL).  RNG streams continue (reset without seed). */
int invsim_reset(invsim_handle *h, const uint8_t *mask, void *obs, void *stream);

/* One Env.step() on all N envs.  actions [N][A]; obs [N][O]; reward [N];
 * terminated/truncated [N]; final_obs [N][O] (SAME_STEP mode only, may be NULL). */
int invsim_step(invsim_handle *h, const void *actions, void *obs, double *reward,
                uint8_t *terminated, uint8_t *truncated, void *final_obs, void *stream);

/* K consecutive steps in one launch (state held in registers between steps):
 * identical results to K invsim_step calls.  actions [K][N][A]; obs [K][N][O];
 * reward/terminated/truncated [K][N]. */
int invsim_rollout(invsim_handle *h, int32_t K, const void *actions, void *obs, double *reward,
                   uint8_t *terminated, uint8_t *truncated, void *stream);

/* Sticky device status word (bit 0: an env was stepped past its horizon with
 * autoreset disabled while the period was not lock-step; such steps are not
 * applied).  Synchronous.  clear != 0 resets it.  invsim_step / invsim_rollout /
 * invsim_rollout_policy of an InvMgmt or NetInvMgmt handle in that state read it
 * themselves (one stream sync) and return INVSIM_ERANGE ("...horizon...") after
 * clearing it: the reference's IndexError (inventory_management.py:267). */
int invsim_status(invsim_handle *h, uint32_t *flags, int32_t clear);

/* ---- Closed-loop rollouts with an in-kernel heuristic agent.
 * The reference's benchmark agents, restated on device:
 *   INVSIM_POLICY_CONSTANT     ConstantOrderAgent  benchmark_NetInvMgmtBacklogEnv.py:119-135
 *                              (any family: the same action every step)
 *   INVSIM_POLICY_BASE_STOCK   BaseStockAgent      benchmark_InvManagementBacklogEnv.py:142-198
 *                              (InvMgmt; also benchmark_InvManagementLostSalesEnv.py:137-165)
 *   INVSIM_POLICY_ORDER_UP_TO  OrderUpToHeuristicAgent  benchmark_newsvendor.py:97-111 (Newsvendor)
 *   INVSIM_POLICY_CLASSIC_NV   ClassicNewsvendorAgent   benchmark_newsvendor.py:113-161 (Newsvendor;
 *                              variant 0 = cr_method 'k_vs_h', 1 = 'profit_margin'; scipy
 *                              poisson.ppf restated on device, newsvendor.hip nv_poisson_ppf)
 *   INVSIM_POLICY_SS           sSPolicyAgent  benchmark_newsvendor_sb3_rllib.py:363-371 (Newsvendor;
 *                              safety_factor carries S_buffer_factor)
 * CLASSIC_NV / SS need mu_max * (lead_time + 1) * max(1, safety_factor) <= 1e6 (INVSIM_ERANGE).
 * Per-env metrics (f64, accumulated with += so a caller may chain launches),
 * the sums evaluate_agent keeps (benchmark_InvManagementBacklogEnv.py:346-440,
 * benchmark_NetInvMgmtLostSalesEnv.py:241-312, benchmark_newsvendor.py:219-250):
 *   [0] sum of rewards (TotalReward)   [1] steps
 *   InvMgmt:    [2] demand_realized  [3] sales[0]  [4] unfulfilled[0]
 *               [5] sum over stages of max(0, ending_inventory)
 *   NetInvMgmt: [2] retail demand D  [3] retail sales S  [4] retail U[t+1]
 *               [5 + j] X[t+1] of main node j (j < n_main)
 *   Newsvendor: [0], [1] only
 * Unavailable with SAME_STEP autoreset and (NetInvMgmt) for graphs other than
 * the reference's default / custom ones (invsim_kernel_variant != 0). */
#define INVSIM_POLICY_CONSTANT 1
#define INVSIM_POLICY_BASE_STOCK 2
#define INVSIM_POLICY_ORDER_UP_TO 3
#define INVSIM_POLICY_CLASSIC_NV 4
#define INVSIM_POLICY_SS 5
#define INVSIM_POLICY_MAX_ACTION 32

typedef struct {
    int32_t kind;            /* INVSIM_POLICY_* */
    int32_t variant;         /* CLASSIC_NV: 0 'k_vs_h', 1 'profit_margin'; else 0 */
    double safety_factor;    /* BASE_STOCK / ORDER_UP_TO / CLASSIC_NV; SS: S_buffer_factor */
    double mu;               /* BASE_STOCK: env.dist_param.get('mu', 10) as the agent reads it */
    const void *constant;    /* CONSTANT: host array [action_dim] in the action dtype */
} invsim_policy;

int invsim_metrics_dim(const invsim_handle *h, int32_t *dim);

/* K steps of every env under `policy`.  All outputs may be NULL: obs [K][N][O],
 * reward / terminated / truncated [K][N], actions [K][N][A] (the actions the
 * agent took), metrics [N][invsim_metrics_dim] (+=).  Autoreset as set. */
int invsim_rollout_policy(invsim_handle *h, int32_t K, const invsim_policy *policy, void *obs, double *reward,
                          uint8_t *terminated, uint8_t *truncated, void *actions, double *metrics, void *stream);

/* Episodic-return statistics of K steps of outputs, the reduction the
 * reference's evaluation harness keeps per episode (episode_rewards ->
 * mean/std, benchmark_InvManagementBacklogEnv.py:389-440).  Handle-free:
 * reward [K][n_envs] f64; terminated / truncated [K][n_envs] u8 (either may be
 * NULL); ret [n_envs] f64 running per-env return (in/out); acc [4] f64 (+=):
 * sum of finished-episode returns, sum of their squares, finished episodes,
 * sum of every reward folded.  Device pointers; the stream's device runs it.
 * invsim.distributed.EpisodeStats all-reduces acc over RCCL. */
int invsim_episode_fold(const double *reward, const uint8_t *terminated, const uint8_t *truncated, int32_t K,
                        int64_t n_envs, double *ret, double *acc, void *stream);

/* The same fold into per-group partials, deterministic (no atomics): part
 * [ceil(n_envs / 64)][4] f64 (+=), row g = [sum of finished-episode returns,
 * sum of their squares, finished episodes, sum of every reward folded] of envs
 * 64 g .. 64 g + 63.  Per env, in row order: ret += reward; at terminated |
 * truncated the return is folded and restarts at 0; each group's per-lane sums
 * over the K rows are then reduced in a fixed order and added to part[g].
 * The statistics are the column sums of part. */
int invsim_episode_fold_groups(const double *reward, const uint8_t *terminated, const uint8_t *truncated,
                               int32_t K, int64_t n_envs, double *ret, double *part, void *stream);

/* Episode sink: the evaluation harness's `episode_reward += reward` per step
 * and its per-episode bookkeeping at done (benchmark_InvManagementBacklogEnv.py:
 * 371, 386, 434), kept on the device inside the step.  With a sink set, every
 * invsim_step / invsim_rollout / invsim_rollout_policy on h folds the rows it
 * produces into ret [N] and part [ceil(N / 64)][4] exactly as
 * invsim_episode_fold_groups over those rows would (same ret and part bits):
 * the lock-step InvMgmt step and rollout kernels in-kernel, other launches by
 * that fold of their outputs on the same stream (reward / terminated /
 * truncated must then be given).  NULL, NULL detaches.  Not during capture. */
int invsim_set_episode_sink(invsim_handle *h, double *ret, double *part);

/* Debug builds only (make -C csrc ptrs_stats -> invsim/_lib/debug/): PTRS
 * log-acceptance statistics since the last clear, summed over kernels:
 * out[0] log tests, out[1] tests ptrs_log_accept's f32 pre-test left to f64,
 * out[2] bit pattern of the smallest relative margin |lhs - rhs| / (sum of
 * |terms|) (f64), out[3] f32-decided tests that disagree with the f64 test,
 * out[4] log tests the decide path's own f32 test (ptrs_decide_d) left to
 * the exact branch (0 in a branchy build).  out has 5 words.  Synchronises the
 * device.  The product build returns INVSIM_EINVAL.  (No reference
 * equivalent: evidence for the numpy random_poisson_ptrs restatement,
 * distributions.c, SURVEY App. B.) */
int invsim_debug_ptrs_stats(uint64_t *out, int32_t clear);

/* Demand stream of a handle.  INVSIM_DEMAND_NUMPY (default): numpy's PCG64
 * Generator stream and samplers, bit-exact with the reference on the same
 * seeds (newsvendor.py:146, inventory_management.py:172,
 * network_management.py:540).  INVSIM_DEMAND_PHILOX: an opt-in, NON-parity
 * fast stream: rocRAND's Philox4x32-10 used counter-based,
 * key = the env's seeded PCG64 increment (high word), counter = (block, draw
 * stream, handle launch step); the same PTRS / multiplication / binomial /
 * integers / geometric transforms.  No per-env generator state is read or
 * written per step.  Every step / rollout step (and a Newsvendor reset)
 * advances the handle's launch-step counter, which get_state / set_state carry
 * ("philox_step"; the first fast-stream call after set_state reads it back,
 * synchronously).  Switching streams synchronises the device (work queued on
 * any stream finishes first); the PCG64 states are untouched by fast-stream
 * steps. */
#define INVSIM_DEMAND_NUMPY 0
#define INVSIM_DEMAND_PHILOX 1
int invsim_set_demand_stream(invsim_handle *h, int32_t mode);
int invsim_demand_stream(const invsim_handle *h, int32_t *mode);

/* Which kernel a handle runs: 0 = the generic kernel of its family, 1 / 2 =
 * NetInvMgmt specialised at compile time for the reference's default /
 * custom supply network (chosen at create when the graph equals one of them). */
int invsim_kernel_variant(const invsim_handle *h, int32_t *variant);

/* Optional per-step demand record (info['demand'] / D): int64 [N][demand_dim],
 * written by every subsequent step/rollout(last step) when non-NULL. */
int invsim_set_info_demand(invsim_handle *h, int64_t *demand);

/* Optional per-step record of the reference's step info (for a single-env
 * view that keeps the reference's history arrays), written by every
 * subsequent step/rollout (last step) when non-NULL:
 *   InvMgmt    int64 [N][2m + 5]:    sales S[t] (m), unfulfilled U[t] (m), then the
 *                                    float64 bit patterns of period_profit, revenue,
 *                                    procurement, holding and penalty cost sums
 *                                    (inventory_management.py:314-345)
 *   NetInvMgmt f64 [N][2 RL + 2 J + 2 E]: S[t, retail links], U[t+1, retail links],
 *                                    X[t+1, main nodes], R[t, reorder links], Y[t+1, reorder
 *                                    links], P[t, main nodes]  (network_management.py:436-619)
 *   Newsvendor f64 [N][5]:          revenue, purchase_cost, holding_cost,
 *                                    lost_sales_penalty (newsvendor.py:149-170, 195-199)
 *                                    and their NumPy-2 kinds packed as
 *                                    k_rev + 4 k_pur + 16 k_hold + 64 k_pen
 *                                    (0 Python float, 1 np.float32, 2 np.float64,
 *                                    3 Python int) */
int invsim_info_record_dim(const invsim_handle *h, int32_t *dim);
int invsim_set_info_record(invsim_handle *h, void *record);

/* Checkpoint / debug: the full device state as one opaque blob of state_bytes,
 * plus a field directory for tests: name, byte offset, element size, rows and
 * row_stride: > 0 rows of row_stride elements ([rows][row_stride]); < 0 a
 * record per env ([-row_stride][rows]); 0 another layout (opaque). */
int invsim_state_bytes(const invsim_handle *h, int64_t *bytes);
int invsim_state_field(const invsim_handle *h, int32_t idx, char name[32], int64_t *offset,
                       int32_t *elem_bytes, int32_t *rows, int64_t *row_stride);
int invsim_get_state(invsim_handle *h, void *dst, void *stream);
int invsim_set_state(invsim_handle *h, const void *src, void *stream);

/* HIP-graph capture of a step loop (SURVEY §7 layer 5; the reference's
 * per-step loop is the caller's `for t: a = agent(obs); env.step(a)`,
 * benchmark_InvManagementBacklogEnv.py:389-440).  The caller records its own
 * stream capture (hipStreamBeginCapture ... hipStreamEndCapture, or
 * torch.cuda.graph) of any mix of its policy launches and invsim_reset /
 * invsim_step / invsim_rollout / invsim_rollout_policy calls on one handle,
 * bracketed by invsim_capture_begin / invsim_capture_end.  Inside the bracket
 * those calls enqueue kernels only; a call that would need a host
 * synchronisation (autoreset DISABLED after a masked reset, get/set_state,
 * status, set_demand_stream) or the fast demand stream (its launch-step
 * counter is a launch parameter and would repeat on replay) fails with
 * INVSIM_EINVAL.  A step call on a capturing stream outside the bracket fails
 * too (the handle's host-side position would drift from the device).
 *
 * The host side of a handle keeps a position (lock-step period, demand
 * lookahead slot) that picks each launch's kernel and parameters.  Nothing
 * runs during capture, so capture_end puts the position back to where
 * capture_begin found it and returns INVSIM_OK only if the captured calls
 * bring it back there (a whole number of episode cycles: periods + 1 steps
 * with NEXT_STEP autoreset, periods with SAME_STEP), so that every replay
 * starts where the graph was recorded; otherwise INVSIM_ERANGE (the graph
 * must not be replayed).  *steps receives the env steps captured.
 * invsim_position returns an opaque token of that position: a graph replays
 * correctly whenever the token equals its value at capture_begin (it does
 * after any number of replays, and after eager calls that close a cycle). */
int invsim_capture_begin(invsim_handle *h);
int invsim_capture_end(invsim_handle *h, int64_t *steps);
int invsim_position(const invsim_handle *h, int64_t *pos);

#ifdef __cplusplus
}
#endif
#endif /* INVSIM_H */
