/*
 * yuma_hip.h — C-ABI of libyuma_hip.so, the MI355X (gfx950) engine for the
 * Yuma consensus epoch step of yuma_simulation.
 *
 * The reference has no FFI: its seam is the Python functions
 *   YumaRust/Yuma/Yuma2/Yuma3/Yuma4(W, S, B_old, config)
 *       src/yuma_simulation/_internal/yumas.py:61,175,285,399,494
 * and the epoch loop that threads the bond state through them
 *   run_simulation(case, yuma_version, yuma_config)
 *       src/yuma_simulation/_internal/simulation_utils.py:26-112
 * The entry points below replace exactly those two seams:
 *   yuma_epoch  <- one call of a Yuma* variant (E = 1, every output optional)
 *   yuma_run    <- the whole epoch loop of run_simulation (E epochs, N scenarios)
 * The Python mirror (yuma_simulation/_internal/engine.py) binds them with
 * ctypes; INTEGRATION.md shows the binding a maintainer adds to the reference.
 *
 * Conventions
 *  - Every pointer argument is DEVICE memory (hipMalloc / torch.cuda tensors),
 *    fp32 row-major, owned by the caller. The engine never allocates, never
 *    synchronises, and is stream-ordered on `stream` (a hipStream_t, NULL =
 *    default stream), so a call can be captured into a hipGraph.
 *  - Layouts: W [E][N][V][M]; S [E][N][V]; B [N][V][M]; per-epoch vectors
 *    [E][N][V] or [E][N][M]; per-epoch matrices [E][N][V][M].
 *  - Return value: 0 on success, a negative YUMA_E* code otherwise;
 *    yuma_last_error() describes the last failure (thread-local).
 */
#ifndef YUMA_HIP_H
#define YUMA_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Variant selector (yumas.py:61 YumaRust, :175 Yuma, :285 Yuma2, :399 Yuma3, :494 Yuma4). */
enum yuma_variant {
  YUMA_VARIANT_RUST = 0,
  YUMA_VARIANT_YUMA1 = 1,
  YUMA_VARIANT_YUMA2 = 2,
  YUMA_VARIANT_YUMA3 = 3,
  YUMA_VARIANT_YUMA4 = 4
};

/* Bond-reset rule applied by run_simulation before an epoch
 * (simulation_utils.py:62-88): Yuma 3.1 resets unconditionally at
 * reset_bonds_epoch; Yuma 3.2 / Yuma 4 only if the previous epoch's
 * consensus of the reset miner is exactly 0. */
enum yuma_reset_mode {
  YUMA_RESET_NONE = 0,
  YUMA_RESET_ALWAYS = 1,
  YUMA_RESET_IF_ZERO_CONSENSUS = 2
};

/* Liquid-alpha modes (yumas.py:231-253 and copies). */
enum yuma_liquid_mode {
  YUMA_LIQUID_OFF = 0,      /* scalar bond_alpha                                 */
  YUMA_LIQUID_QUANTILE = 1, /* consensus high/low from quantiles (or one override) */
  YUMA_LIQUID_CONST_AB = 2  /* both overrides given and unequal: a,b host doubles */
};

enum yuma_override_flags { YUMA_OVR_HIGH = 1, YUMA_OVR_LOW = 2, YUMA_OVR_FORCE_Q99 = 4 };

/* yuma_params_t.flags. YUMA_FLAG_NO_HIST: run the consensus search as the
 * plain bisection even where the exact-stake histogram finish applies (both
 * give the same result; tests compare them). YUMA_FLAG_RESET_ALL_COLUMNS: the
 * reset zeroes every miner column (reset_index ignored) -- the reference's
 * `B_state[:, None] = 0.0` when reset_bonds_index is None
 * (simulation_utils.py:63-64). */
enum yuma_flags { YUMA_FLAG_NO_HIST = 1, YUMA_FLAG_RESET_ALL_COLUMNS = 2 };

/* Per-scenario parameters: the flattened YumaConfig (yumas.py:7-45) with every
 * Python-double constant pre-rounded exactly as the reference's torch ops round
 * them (python scalars meet fp32 tensors as fp32). 128 bytes, naturally aligned. */
typedef struct yuma_params {
  int32_t variant;          /* yuma_variant (must equal the call's variant)        */
  int32_t bisect_iters;     /* trip count of `while (hi-lo) > 1/consensus_precision` */
  int32_t liquid_mode;      /* yuma_liquid_mode                                    */
  int32_t override_flags;   /* yuma_override_flags                                 */
  int32_t reset_mode;       /* yuma_reset_mode                                     */
  int32_t reset_epoch;      /* epoch index of the reset (run_simulation epoch)     */
  int32_t reset_index;      /* miner column to reset, 0 <= reset_index < M         */
  int32_t flags;            /* yuma_flags                                          */
  float kappa;              /* fp32(kappa)                                         */
  float bond_penalty;       /* fp32(beta)                                          */
  float one_minus_bond_penalty; /* fp32(1 - beta), difference taken in double      */
  float bond_alpha;         /* fp32(bond_alpha)                                    */
  float one_minus_bond_alpha;   /* fp32(1 - bond_alpha), difference in double      */
  float alpha_low;          /* fp32(alpha_low)                                     */
  float alpha_high;         /* fp32(alpha_high)                                    */
  float capacity_alpha;     /* fp32(capacity_alpha)           (Yuma3)              */
  float decay_keep;         /* fp32(1 - decay_rate)           (Yuma3)              */
  float maxint;             /* fp32(maxint) = 2^64 for the default (Yuma3)         */
  float const_a;            /* LIQUID_CONST_AB: fp32(a)                            */
  float const_b;            /* LIQUID_CONST_AB: fp32(b)                            */
  double ln_num;            /* log(1/alpha_high-1) - log(1/alpha_low-1)             */
  double ln_low;            /* log(1/alpha_low-1)                                  */
  double override_high;     /* override_consensus_high (if flagged)                */
  double override_low;      /* override_consensus_low (if flagged)                 */
  double reserved1[2];
} yuma_params_t;

/* Optional outputs; any pointer may be NULL (not produced). The dict keys of
 * the reference (yumas.py:264-282 etc.) are noted per field. */
typedef struct yuma_outputs {
  float* Dn;         /* [E][N][V] validator_reward_normalized                    */
  float* D;          /* [E][N][V] validator_reward                               */
  float* C;          /* [E][N][M] server_consensus_weight (quantised)            */
  float* I;          /* [E][N][M] server_incentive                               */
  float* R;          /* [E][N][M] server_rank                                    */
  float* P;          /* [E][N][M] server_prerank                                 */
  float* T;          /* [E][N][M] server_trust                                   */
  float* Tv;         /* [E][N][V] validator_trust                                */
  float* Sn;         /* [E][N][V] stake (normalised)                             */
  float* bond_alpha; /* [E][N][M] liquid bond_alpha per miner (liquid only)      */
  float* alpha_ab;   /* [E][N][2] alpha_a, alpha_b (liquid only)                 */
  float* Wn;         /* [E][N][V][M] weight (row-normalised)                     */
  float* Wc;         /* [E][N][V][M] consensus_clipped_weight                    */
  float* Wb;         /* [E][N][V][M] weight_for_bond (Yuma1/Yuma2)               */
  float* B_inst;     /* [E][N][V][M] validator_bond (Rust/Yuma1/Yuma2)           */
  float* B_hist;     /* [E][N][V][M] bond state after each epoch (bonds_per_epoch) */
  float* B_final;    /* [N][V][M]    bond state after the last epoch             */
} yuma_outputs_t;

enum {
  YUMA_OK = 0,
  YUMA_EINVAL = -1,    /* bad sizes / pointers / params                          */
  YUMA_EWORKSPACE = -2,/* workspace too small                                    */
  YUMA_EHIP = -3,      /* a HIP launch failed                                    */
  YUMA_EUNSUPPORTED = -4
};

/* Validators per slice. Up to YUMA_REG_VALIDATORS a workgroup holds a miner
 * column's validators in registers (the fast paths); above, the engine streams
 * the column from memory in every consensus pass and runs YumaRust's bond
 * normalisation as two launches per epoch (correct at any size up to
 * YUMA_MAX_VALIDATORS, built for the occasional very wide validator set). */
#define YUMA_REG_VALIDATORS 1024
#define YUMA_MAX_VALIDATORS (1 << 20)

/* Bytes of device workspace yuma_run / yuma_epoch need for these sizes.
 * full_outputs != 0 reserves the partial sums the validator_trust output
 * (yuma_outputs_t.Tv) needs; without it a non-NULL Tv is rejected.        */
size_t yuma_workspace_bytes(int variant, int N, int E, int V, int M, int full_outputs);

/* The whole epoch loop of run_simulation (simulation_utils.py:44-110) for N
 * independent scenarios of one variant, E epochs each.
 *   params_dev : [N] yuma_params_t in device memory
 *   W          : [E][N][V][M] raw weights (row-normalised inside, yumas.py:186)
 *   S          : [E][N][V] raw stakes (normalised inside, yumas.py:189)
 *   B_init     : [N][V][M] bond state before epoch 0, or NULL (= B_state None)
 *   Wprev_init : Yuma2 only: [N][V][M] normalised W_prev for epoch 0, or NULL
 *   chunk_epochs: epochs per phase-1 batch (0 = engine default)                */
int yuma_run(int variant, const yuma_params_t* params_dev, int N, int E, int V, int M,
             const float* W, const float* S, const float* B_init, const float* Wprev_init,
             const yuma_outputs_t* out, void* workspace, size_t workspace_bytes,
             int chunk_epochs, void* stream);

/* yuma_run with options. flags: YUMA_RUN_SHARED_INPUTS — every scenario reads
 * the same input trajectory: W is [E][V][M] and S [E][V] (a parameter sweep
 * over one subnet; SURVEY config c3), so a whole sweep moves one copy of W
 * per epoch through HBM and the scenarios' reads of it meet in the caches.
 * Results are those of yuma_run on W and S replicated per scenario.
 * phase_ms: NULL, or per-phase device time as yuma_run_profiled (blocks).   */
enum yuma_run_flags { YUMA_RUN_SHARED_INPUTS = 1 };
int yuma_run_ex(int variant, const yuma_params_t* params_dev, int N, int E, int V, int M,
                const float* W, const float* S, const float* B_init, const float* Wprev_init,
                const yuma_outputs_t* out, void* workspace, size_t workspace_bytes,
                int chunk_epochs, int flags, void* stream, float* phase_ms);

/* hipGraph form of yuma_run: the whole multi-epoch run (every phase of every
 * chunk, no host work between them) captured once into a HIP graph and
 * replayed with one hipGraphLaunch. The arguments are those of yuma_run and
 * are baked into the graph: every replay reads the same W / S / params /
 * B_init buffers (refill them in place between replays) and writes the same
 * outputs. Capture happens on an internal stream; `stream` orders the capture
 * after the caller's prior work only through the caller's own sync, so call
 * it with inputs already resident. Replaces the per-epoch Python loop of
 * run_simulation (simulation_utils.py:52-110) for repeated runs.            */
typedef struct yuma_graph* yuma_graph_t;
int yuma_graph_create(yuma_graph_t* graph, int variant, const yuma_params_t* params_dev, int N,
                      int E, int V, int M, const float* W, const float* S,
                      const float* B_init, const float* Wprev_init, const yuma_outputs_t* out,
                      void* workspace, size_t workspace_bytes, int chunk_epochs);
/* yuma_graph_create with yuma_run_ex's flags. */
int yuma_graph_create_ex(yuma_graph_t* graph, int variant, const yuma_params_t* params_dev, int N,
                         int E, int V, int M, const float* W, const float* S,
                         const float* B_init, const float* Wprev_init, const yuma_outputs_t* out,
                         void* workspace, size_t workspace_bytes, int chunk_epochs, int flags);
/* Replay on `stream` (stream-ordered, no host synchronisation). */
int yuma_graph_launch(yuma_graph_t graph, void* stream);
/* Kernel nodes in the captured graph (diagnostics / tests). */
int yuma_graph_nodes(yuma_graph_t graph);
int yuma_graph_destroy(yuma_graph_t graph);

/* Phases of a run, in launch order (per chunk of epochs). */
enum yuma_phase {
  YUMA_PHASE_ROWSUM = 0,    /* k_rowsum:    row sums, stake normalisation      */
  YUMA_PHASE_CONSENSUS = 1, /* k_consensus: bisection per miner column          */
  YUMA_PHASE_QUANTISE = 2,  /* k_quantise:  C quantisation, liquid alpha        */
  YUMA_PHASE_RANK = 3,      /* k_rank:      clip, rank                          */
  YUMA_PHASE_INCENTIVE = 4, /* k_incentive: incentive, trust                    */
  YUMA_PHASE_BONDS = 5,     /* k_bonds:     bond recurrence over the chunk      */
  YUMA_PHASE_FINALIZE = 6,  /* k_finalize:  dividends                           */
  YUMA_NUM_PHASES = 7
};

/* yuma_run plus per-phase device time: HIP events are recorded on `stream`
 * between phases and phase_ms[YUMA_NUM_PHASES] receives the milliseconds
 * spent in each phase summed over chunks. Blocks until
 * the stream reaches the end of the run. For benchmarks / roofline only. */
int yuma_run_profiled(int variant, const yuma_params_t* params_dev, int N, int E, int V, int M,
                      const float* W, const float* S, const float* B_init,
                      const float* Wprev_init, const yuma_outputs_t* out, void* workspace,
                      size_t workspace_bytes, int chunk_epochs, void* stream, float* phase_ms);

/* One call of a Yuma* variant for N independent slices (E = 1):
 * yumas.py:61 (YumaRust), :175 (Yuma), :285 (Yuma2, W_prev may be NULL),
 * :399 (Yuma3), :494 (Yuma4). B_old may be NULL (first epoch).             */
int yuma_epoch(int variant, const yuma_params_t* params_dev, int N, int V, int M,
               const float* W, const float* W_prev, const float* S, const float* B_old,
               const yuma_outputs_t* out, void* workspace, size_t workspace_bytes,
               void* stream);

/* ------------------------------------------------------------------------
 * Miner-column sharding of one wide subnet.
 *
 * The reference runs a wide subnet as one Yuma* call per epoch
 * (yumas.py:399 etc., driven by run_simulation, simulation_utils.py:44-110).
 * Every cross-miner quantity of that epoch step is a sum over miner columns
 * (row sums :186, sum C :211, sum R :220, D :261/:474/:589) or a quantile of
 * C (:231-247), and the bond recurrence is column-local, so a process can own
 * columns [col0, col0 + M) of an M_total-wide subnet. yuma_shard_stage runs
 * stage k of the whole E-epoch run on those columns; between stages the
 * caller combines the per-shard partials of every shard (RCCL all-gather,
 * summed in shard order) and hands the totals back through `io`:
 *
 *   stage 1 -> rowsum_part [E][N][V] = sum over local columns of W
 *   stage 2 <- rowsum      [E][N][V] = sum over shards of rowsum_part
 *           -> csum_part   [E][N]    = sum of local C_raw (fp32; YumaRust:
 *                                      csum_part_d, fp64)
 *   stage 3 <- csum / csum_d [E][N]
 *           -> levels      [E][N][M] quantisation levels of local columns
 *              rsum_part   [E][N]    = sum of local R
 *   stage 4 <- rsum [E][N]; levels_all [E][N][M_total] (liquid scenarios)
 *           -> dsum_part   [E][N][V] = sum over local columns of B * I
 *   stage 5 <- dsum [E][N][V]; writes Dn / D
 * validator_trust (out->Tv, yumas.py:224 `W_clipped.sum(1) / W.sum(1)`):
 *   stage 3 -> tv_part [2][E][N][V] = sums over local columns of Wc and Wn
 *   stage 5 <- tv      [2][E][N][V] = sum over shards of tv_part; Tv = tv[0] / tv[1]
 *   (the workspace must then be sized with full_outputs = 1)
 *
 * Every stage takes the same arguments as yuma_run (W [E][N][V][M] holds the
 * local columns; outputs are the local columns of the [..][M] outputs) and
 * the same workspace, which carries state from stage to stage. params must
 * carry reset_index relative to col0 (reset_mode NONE on shards that do not
 * own the reset column).
 * ---------------------------------------------------------------------- */
typedef struct yuma_shard_io {
  int M_total;             /* global miner count                              */
  int col0;                /* first global column held by this shard          */
  float* rowsum_part;      /* stage 1 out                                     */
  const float* rowsum;     /* stage 2 in                                      */
  float* csum_part;        /* stage 2 out (not YumaRust)                      */
  double* csum_part_d;     /* stage 2 out (YumaRust)                          */
  const float* csum;       /* stage 3, 4 in (not YumaRust)                    */
  const double* csum_d;    /* stage 3, 4 in (YumaRust)                        */
  int* levels;             /* stage 3 out                                     */
  float* rsum_part;        /* stage 3 out                                     */
  const float* rsum;       /* stage 4 in                                      */
  const int* levels_all;   /* stage 4 in, required when a scenario is liquid  */
  float* dsum_part;        /* stage 4 out                                     */
  const float* dsum;       /* stage 5 in                                      */
  float* tv_part;          /* stage 3 out when out->Tv: [2][E][N][V]          */
  const float* tv;         /* stage 5 in when out->Tv:  [2][E][N][V]          */
} yuma_shard_io_t;

int yuma_shard_stage(int stage, int variant, const yuma_params_t* params_dev, int N, int E,
                     int V, int M, const float* W, const float* S, const float* B_init,
                     const float* Wprev_init, const yuma_shard_io_t* io,
                     const yuma_outputs_t* out, void* workspace, size_t workspace_bytes,
                     void* stream);

/* Deterministic synthetic inputs: integer-valued weights whose
 * row sums are exact in fp32. Writes W[e][n][v][m] for epochs t0..t0+E-1.
 * Bit-identical to yuma_simulation._internal.synth.weights (numpy).          */
int yuma_synth_weights(uint64_t seed, int E, int N, int V, int M, int t0, float* W,
                       void* stream);

const char* yuma_last_error(void);
const char* yuma_version(void);
/* Build identity of this library: "src-" + the first 16 hex digits of the
 * SHA-256 of the engine source and this header it was compiled from (stamped
 * by __graft_entry__.build / tools/ab_build.py; "unstamped" otherwise).
 * bench.py pairs a committed counter record with a run only when their build
 * ids match (no reference counterpart: measurement plumbing).               */
const char* yuma_build_id(void);

#ifdef __cplusplus
}
#endif
#endif /* YUMA_HIP_H */
