/*
 * ldpc_mi355x.h -- C ABI of libldpc_mi355x.so, the MI355X (gfx950) LDPC
 * belief-propagation engine.
 *
 * Plain C types only (pointers + sizes); no torch / HIP types in signatures.
 * `stream` arguments are hipStream_t passed as void* (NULL = default stream).
 *
 * Every entry point cites the reference interface it replaces or extends
 * (paths relative to roryhighnam/iib_project_ldpc_codes).
 *
 * Return convention for the new entry points: 0 = OK, negative = error
 * (LDPC_E*); ldpc_last_error() returns a human-readable message.  The drop-in
 * message_passing keeps the reference's convention (returns the iteration
 * index) and returns a negative LDPC_E* code on failure.
 *
 * Empty batches: B = 0 is a no-op returning LDPC_OK (after the graph and
 * shape checks); the per-codeword buffers may then be NULL (an empty device
 * tensor's data pointer).  max_iters = 0: BEC words are left as they are with
 * its = 0; soft decoders return the channel LLRs as posteriors.
 */
#ifndef LDPC_MI355X_H
#define LDPC_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDPC_OK 0
#define LDPC_EINVAL (-1)  /* bad argument / inconsistent graph / value outside {0,1,2} */
#define LDPC_ENODEV (-2)  /* no MI355X visible / HIP runtime error at init */
#define LDPC_EHIP (-3)    /* HIP runtime error during a call */
#define LDPC_ENOMEM (-4)
#define LDPC_EUNSUP (-5)  /* configuration not supported by any kernel */

/* Channels (channels.py:4-26 BEC; BSC and BI-AWGN are new). */
#define LDPC_CH_BEC 0   /* param = erasure probability                          */
#define LDPC_CH_BSC 1   /* param = crossover probability                        */
#define LDPC_CH_AWGN 2  /* param = noise std-dev sigma (BPSK +-1, LLR = 2y/s^2)  */

/* Soft decoding algorithms (no reference counterpart). */
#define LDPC_ALGO_SPA 0      /* sum-product, tanh rule, fp32                     */
#define LDPC_ALGO_MINSUM 1   /* normalized min-sum (alpha), fp32                 */

/* ---------------------------------------------------------------------- */
/* Drop-in                                                                 */
/* ---------------------------------------------------------------------- */
/*
 * Replaces message_passing.c:7 (`int message_passing(int *Mvc, int iterations,
 * int *variable_to_check_list, int *check_to_variable_list, int *errors, int n,
 * int k, int dv, int dc)`), bound by ctypes at parallel_simulator.py:162-164
 * and parallel_simulator_expurgated.py:162-164.  Same symbol, arguments and
 * semantics: Mvc (0/1/2, int32[n]) decoded in place, errors[it] += erasure
 * count per iteration (caller zeroes it), stall skip, returns the break
 * iteration or `iterations`.  Runs one codeword on the current HIP device.
 * Per call: the lists are compared with the last call's (exact memcmp) and the
 * cached device graph reused, or refilled in place for a new code of the same
 * shape; the word and errors[] travel through pinned staging, one copy each
 * way, one stream synchronisation (thread-safe; one cache per process).
 */
int message_passing(int *Mvc, int iterations, int *variable_to_check_list,
                    int *check_to_variable_list, int *errors, int n, int k, int dv, int dc);

/* ---------------------------------------------------------------------- */
/* Tanner graph handle                                                     */
/* ---------------------------------------------------------------------- */
typedef struct ldpc_graph ldpc_graph;

/*
 * Upload a regular graph given in the reference's edge-list format
 * (random_code_generator.c:34-36 check_lookup = check_to_variable_list,
 * int32[(n-k)*dc]; random_code_generator.c:57-62 variable_lookup =
 * variable_to_check_list, int32[n*dv]) to the current device.
 */
int ldpc_graph_create(const int32_t *variable_to_check_list, const int32_t *check_to_variable_list,
                      int n, int k, int dv, int dc, ldpc_graph **out);

/*
 * Upload an irregular graph in CSR slot form (new):
 * check c owns slots [check_ptr[c], check_ptr[c+1]) with check_var[slot] its
 * variable; variable v owns edges [var_ptr[v], var_ptr[v+1]) with var_slot[]
 * naming the slot of each edge.
 */
int ldpc_graph_create_csr(const int32_t *check_ptr, const int32_t *check_var, const int32_t *var_ptr,
                          const int32_t *var_slot, int n, int m, ldpc_graph **out);

void ldpc_graph_destroy(ldpc_graph *g);
int ldpc_graph_info(const ldpc_graph *g, int32_t *n, int32_t *m, int32_t *num_edges);

/* ---------------------------------------------------------------------- */
/* Batched BEC erasure decoding (message_passing.c:7-82 over B words)     */
/* ---------------------------------------------------------------------- */
/*
 * Host-pointer form: words uint8[B*n] (0/1/2, in/out),
 * errors int32[B*max_iters] (accumulated, as message_passing.c:73),
 * its int32[B] (return value of each message_passing call).
 */
int ldpc_bec_decode_batch(const int32_t *variable_to_check_list, const int32_t *check_to_variable_list,
                          int n, int k, int dv, int dc, uint8_t *words, int B, int max_iters,
                          int32_t *errors, int32_t *its);

/* Device-pointer form on a prepared graph; asynchronous on `stream`. */
int ldpc_bec_decode_batch_dev(const ldpc_graph *g, uint8_t *d_words, int B, int max_iters,
                              int32_t *d_errors, int32_t *d_its, void *stream);

/* ---------------------------------------------------------------------- */
/* Batched soft decoding (new: SURVEY.md 8b-3)                            */
/* ---------------------------------------------------------------------- */
/*
 * llr float[B*n] channel LLRs (log P(0)/P(1)); outputs posterior LLRs
 * post float[B*n] (may be NULL), hard decisions hard uint8[B*n] (may be NULL,
 * 1 where post < 0) and iterations run its int32[B] (may be NULL).
 * early_stop != 0 stops a codeword once its hard decision satisfies every check.
 * With early stop and post == NULL only the stopping iteration's decisions and
 * the iteration counts are produced, which lets the decode run on the
 * local-edge kernel (same decisions and counts as the posterior-returning path).
 */
int ldpc_bp_decode_batch(const int32_t *variable_to_check_list, const int32_t *check_to_variable_list,
                         int n, int k, int dv, int dc, const float *llr, int B, int max_iters,
                         int algo, float alpha, int early_stop, float *post, uint8_t *hard,
                         int32_t *its);

int ldpc_bp_decode_batch_dev(const ldpc_graph *g, const float *d_llr, int B, int max_iters, int algo,
                             float alpha, int early_stop, float *d_post, uint8_t *d_hard,
                             int32_t *d_its, void *stream);

/* ---------------------------------------------------------------------- */
/* On-device channels (channels.py:24-26 new_transmit + BSC / BI-AWGN)     */
/* ---------------------------------------------------------------------- */
/*
 * Channel outputs for the all-zero codeword (parallel_simulator.py:222) of
 * codewords first_cw .. first_cw+B-1, Philox4x32-10 (rocRAND) keyed by seed:
 * BEC writes uint8 0/2 into d_out, BSC / AWGN write float LLRs.
 */
int ldpc_channel_dev(int channel, float param, uint64_t seed, uint64_t first_cw, int n, int B,
                     void *d_out, void *stream);

/* ---------------------------------------------------------------------- */
/* Monte-Carlo batch (run_simulation trial loop, parallel_simulator.py:198-244) */
/* ---------------------------------------------------------------------- */
/*
 * One fused device batch: B trials first_cw .. first_cw+B-1: channel ->
 * decode -> per-trial statistics.  counters int64[LDPC_MC_NCOUNT + max_iters + 1]
 * on the device, ACCUMULATED (+=):
 *   [0] trials  [1] frame errors  [2] bit errors (residual erasures / wrong bits)
 *   [3] decoding iterations executed  [4..] error curve[0..max_iters]
 *   (BEC: erasures before decoding and after each iteration -- the
 *    `errors` vector of parallel_simulator.py:165 summed as at :227;
 *    soft: wrong hard decisions after each iteration, [4] = channel errors).
 * A trial counts only when its final error count is > expurgation
 * (parallel_simulator_expurgated.py:238); pass -1 for the plain simulator.
 * If stop_frame_errors > 0 the batch honours the sequential stop rule
 * (parallel_simulator.py:198): only trials up to and including the one that
 * brings counters[1] to stop_frame_errors are counted.
 * algo is ignored for BEC (exact erasure decoding, message_passing.c).
 */
#define LDPC_MC_NCOUNT 4
int ldpc_mc_batch_dev(const ldpc_graph *g, int channel, float param, uint64_t seed, uint64_t first_cw,
                      int B, int max_iters, int algo, float alpha, int early_stop, int expurgation,
                      int64_t stop_frame_errors, int64_t *d_counters, void *stream);

/* ---------------------------------------------------------------------- */
/* Whole Monte-Carlo run over several devices of one process */
/* ---------------------------------------------------------------------- */
/*
 * Replaces the trial loop of run_simulation / run_simulation_fixed_ldpc
 * (parallel_simulator.py:198-244, :354-379; parallel_simulator_expurgated.py
 * :200-256) together with the reference's multi-process fan-out
 * (parallel_simulator.py:403-445) and CSV merge (tools/combine_data.py:64-95):
 * one call runs `while frame_errors < stop_frame_errors and trials < num_tests`
 * (either limit <= 0 = none; time_limit_s <= 0 = none, else checked after each
 * round) over devices[0..ndev) (HIP ordinals, each listed once).  Device slot r
 * of round R decodes trials [(R*ndev + r)*batch, +batch); the counters of each
 * round are summed with ONE ncclAllReduce over the devices (RCCL,
 * ncclCommInitAll, loaded from librccl.so.1 at first use).  The stop rule is
 * applied exactly in global trial order, so the result equals one sequential
 * process over the same trials whatever ndev is.
 *   Graph: the reference's edge lists (fixed code, built on every device) -- or
 *   both lists NULL for ensemble mode (a fresh random (dv, dc) code per trial,
 *   BEC only, parallel_simulator.py:215); ldpc_mc_run_csr takes a CSR graph
 *   (irregular codes).
 *   counters (host) int64[LDPC_MC_NCOUNT + max_iters + 1], layout as
 *   ldpc_mc_batch_dev, overwritten; rounds (may be NULL) = rounds run.
 */
int ldpc_mc_run(const int32_t *variable_to_check_list, const int32_t *check_to_variable_list, int n, int k,
                int dv, int dc, int channel, float param, int algo, float alpha, int early_stop, uint64_t seed,
                int max_iters, int expurgation, int64_t num_tests, int64_t stop_frame_errors, int batch,
                double time_limit_s, const int *devices, int ndev, int64_t *counters, int64_t *rounds);
int ldpc_mc_run_csr(const int32_t *check_ptr, const int32_t *check_var, const int32_t *var_ptr,
                    const int32_t *var_slot, int n, int m, int channel, float param, int algo, float alpha,
                    int early_stop, uint64_t seed, int max_iters, int expurgation, int64_t num_tests,
                    int64_t stop_frame_errors, int batch, double time_limit_s, const int *devices, int ndev,
                    int64_t *counters, int64_t *rounds);

/* ---------------------------------------------------------------------- */
/* Random regular graphs + ensemble Monte-Carlo           */
/* ---------------------------------------------------------------------- */
/*
 * Replaces generate_random_code (random_code_generator.c:21-67, called per
 * trial at parallel_simulator.py:215 / parallel_simulator_expurgated.py:221-223):
 * G graphs first_graph .. first_graph+G-1 of the (dv, dc) configuration model
 * with whole-graph redraw while any check holds a variable twice, in the
 * reference's edge-list format: check_lookup int32[G][n*dv] (variables of check
 * c at [c*dc, c*dc+dc)), variable_lookup int32[G][n*dv] (checks of each variable,
 * ascending).  Counter-based (Philox, key = seed): graph g is the same whatever
 * G / first_graph batch it is drawn in.  attempts int32[G] (may be NULL): number
 * of permutations drawn for each graph.  The dense parity-check matrix is never
 * built.
 */
int ldpc_sample_regular_dev(int n, int dv, int dc, uint64_t seed, uint64_t first_graph, int G,
                            int32_t *d_check_lookup, int32_t *d_variable_lookup, int32_t *d_attempts,
                            void *stream);
int ldpc_sample_regular(int n, int dv, int dc, uint64_t seed, uint64_t first_graph, int G,
                        int32_t *check_lookup, int32_t *variable_lookup, int32_t *attempts);

/*
 * Irregular form (the same law for any degree structure): n
 * variables with var_ptr[v+1]-var_ptr[v] sockets each, m checks with
 * check_ptr[c+1]-check_ptr[c] slots each (host arrays, var_ptr[n] ==
 * check_ptr[m] == E); a uniformly random socket->slot matching, redrawn whole
 * while any check holds a variable twice.  Output per graph g (row-major):
 * check_var int32[G][E] (variable of each slot, check-major) and var_slot
 * int32[G][E] (for variable v, entries var_ptr[v].. = its slots ascending) --
 * the ldpc_graph_create_csr layout.  Same generator as ldpc_sample_regular
 * (which is this with var_ptr = v*dv, check_ptr = c*dc, var_slot -> check ids).
 */
int ldpc_sample_csr_dev(int n, int m, const int32_t *var_ptr, const int32_t *check_ptr, uint64_t seed,
                        uint64_t first_graph, int G, int32_t *d_check_var, int32_t *d_var_slot, int32_t *d_attempts,
                        void *stream);
int ldpc_sample_csr(int n, int m, const int32_t *var_ptr, const int32_t *check_ptr, uint64_t seed,
                    uint64_t first_graph, int G, int32_t *check_var, int32_t *var_slot, int32_t *attempts);

/*
 * Ensemble BEC Monte-Carlo batch (run_simulation, parallel_simulator.py:168-272;
 * expurgated :169-285): trial t = first_cw + b draws graph t and channel word t,
 * decodes with message_passing semantics and accumulates counters exactly as
 * ldpc_mc_batch_dev (expurgation, sequential stop rule).
 */
int ldpc_mc_ensemble_batch_dev(int n, int dv, int dc, int channel, float param, uint64_t seed,
                               uint64_t first_cw, int B, int max_iters, int expurgation,
                               int64_t stop_frame_errors, int64_t *d_counters, void *stream);

/* ---------------------------------------------------------------------- */
/* ML ("optimal") erasure decoding                        */
/* ---------------------------------------------------------------------- */
/*
 * Replaces regular_LDPC_code.optimal_decode (parallel_simulator.py:60-129;
 * expurgated :60-129) together with the ml_decode set-up it calls through ctypes
 * (ml_decoder.c:7-36, bound at parallel_simulator.py:83-84) and the GF(2)
 * row_reduce of the galois package (:89-91, :108).  Words are uint8 [B][n]:
 * 0/1 known bits, 2 erasures (any other non-zero value is a known 1 and is
 * returned as given).  Output: the decoded words, 2 where an unknown was given up
 * by the reference's loop (first non-pivot column dropped with all its checks,
 * system reduced again); words with no erasure or more erasures than n-k are
 * returned unchanged.  unsolved int32 [B] = the number of 2s in each output word
 * (the reference's optimal_error_count, :235).  d_out may alias d_words.
 * Needs m = n-k <= 1000 (the range in which the reference's 1000-unknown cap,
 * :96, never binds) and n <= 32767; otherwise LDPC_EINVAL.
 */
int ldpc_ml_decode_batch_dev(const ldpc_graph *g, const uint8_t *d_words, int B, uint8_t *d_out,
                             int32_t *d_unsolved, void *stream);
int ldpc_ml_decode_batch(const ldpc_graph *g, const uint8_t *words, int B, uint8_t *out, int32_t *unsolved);

/* Ensemble form: word b is decoded on graph b of d_check_lookup int32[B][n*dv]
 * (the ldpc_sample_regular_dev output layout). */
int ldpc_ml_ensemble_decode_dev(int n, int dv, int dc, const int32_t *d_check_lookup, const uint8_t *d_words, int B,
                                uint8_t *d_out, int32_t *d_unsolved, void *stream);

/*
 * Monte-Carlo batch of the "optimal" modes 1/2/4/5 (parallel_simulator.py:
 * 168-272 / 274-401, `optimal` = True): BEC(eps) channel word t = first_cw + b,
 * ML-decoded; with message_passing != 0 the same word is also BEC-decoded for
 * max_iters iterations (modes 2/5).  g == NULL: ensemble mode, trial t decodes on
 * graph t of the (n, dv, dc) sampler (ldpc_sample_regular law, key = seed);
 * otherwise n/dv/dc are ignored.  d_counters_ml int64[LDPC_MC_NCOUNT + 1] =
 * [trials, ML frame errors, ML bit errors (# of 2s), 0, # of 2s];
 * d_counters_mp int64[LDPC_MC_NCOUNT + max_iters + 1] as ldpc_mc_batch_dev
 * (expurgation applies to it only, as parallel_simulator_expurgated.py:238-245).
 * The sequential stop rule counts message-passing frame errors when
 * message_passing != 0, ML frame errors otherwise (parallel_simulator.py:186-242).
 */
int ldpc_mc_ml_batch_dev(const ldpc_graph *g, int n, int dv, int dc, float eps, uint64_t seed, uint64_t first_cw,
                         int B, int max_iters, int message_passing, int expurgation, int64_t stop_frame_errors,
                         int64_t *d_counters_mp, int64_t *d_counters_ml, void *stream);

/* ---------------------------------------------------------------------- */
/* Diagnostics (host only, no GPU needed)                                  */
/* ---------------------------------------------------------------------- */
/*
 * The conflict-aware lane layout the LDS-resident soft kernel uses for this
 * graph: *T threads x *VPT variables per thread; lane_var int32[T*VPT]
 * (-1 = padding), lane_slot int32[T*VPT*dv].  Pass NULL arrays to query T/VPT.
 */
int ldpc_debug_lane_layout(const int32_t *variable_to_check_list, const int32_t *check_to_variable_list,
                           int n, int k, int dv, int dc, int32_t *T, int32_t *VPT, int32_t *lane_var,
                           int32_t *lane_slot);

/*
 * The irregular kernel's layout for a consistent CSR graph (ldpc_graph_create_csr
 * arguments): shape[5] = {VPT, KC (check rows of 1024), DC (slots per check),
 * S (positions in LDS), P (positions in all)}; lane int32[3][1024*VPT] (variable
 * id or -1, positions of edges 0|1<<16 and 2|3<<16, 0xFFFF = none); cdeg
 * int32[2][1024] (check degrees, 4 bits per row).  Returns LDPC_EUNSUP when the
 * graph is outside the kernel's range.  Pass NULL arrays to query the shape.
 */
int ldpc_debug_irr_layout(const int32_t *check_ptr, const int32_t *check_var, const int32_t *var_ptr,
                          const int32_t *var_slot, int n, int m, int32_t *shape, int32_t *lane, int32_t *cdeg);

/*
 * Host-only: the local-edge layout of bp_loc_kernel for a CSR graph (no device
 * needed; tests / diagnostics).  shape: int32[24] = {T, KP, DVN, P, words, classes,
 * bank-conflict cost, cls_q[5], cls_d[4], cls_w[5], DVN0 | ABS0 << 8, DVN1 | ABS1 << 8}; var: int32[2*KP*2*T] variable
 * ids, pos: int32[2*KP*max(DVN,1)*T] packed LDS words, info: int32[2*KP*T] (see
 * ldpc_graph::loc_* in csrc/ldpc_internal.hpp).  NULL arrays: shape only.  Returns
 * LDPC_EUNSUP when the graph has no such layout.
 */
int ldpc_debug_loc_layout(const int32_t *check_ptr, const int32_t *check_var, const int32_t *var_ptr,
                          const int32_t *var_slot, int n, int m, int T, int32_t *shape, int32_t *var, int32_t *pos,
                          int32_t *info);

/*
 * Host-only: ldpc_mc_run's round accounting (csrc/mc_plan.hpp: per-slot batch clamp to
 * num_tests, the crossing slot's cut at its share of the remaining frame errors, later slots
 * dropped) driven by the same loop as the device run, on a synthetic trial sequence:
 * trial t is a frame error iff frame_error[t] != 0 (t < num_trials).  out int64[3] = {trials,
 * frame errors, rounds} -- equal to the sequential `while frame_errors < stop and trials <
 * num_tests` loop (parallel_simulator.py:198) for every ndev.  LDPC_EINVAL if the plan would
 * read past num_trials.
 */
int ldpc_debug_mc_plan(const uint8_t *frame_error, int64_t num_trials, int64_t num_tests, int64_t stop_frame_errors,
                       int batch, int ndev, int64_t *out);

/*
 * Host-only: which bp_loc_kernel instantiation family the local-edge layout of this CSR
 * graph (at T threads) would run on: 0 none (the graph takes another soft kernel), 1 the
 * (3,6) family <6,6,2,2> (every check degree 6, every variable degree 3), 2 the RSU family
 * <5,6,1,3> (check degrees 5..6, slot-0 variables degree 2, others 2..4).  Decided from the
 * whole layout shape, exactly as the device dispatch decides it.
 */
int ldpc_debug_loc_variant(const int32_t *check_ptr, const int32_t *check_var, const int32_t *var_ptr,
                           const int32_t *var_slot, int n, int m, int T, int32_t *variant);

/*
 * Device diagnostics: the sequential-draw sampler's counters accumulated since the last reset,
 * out uint64[32]: the search pass's 16 (attempts, aborted attempts, rounds, slots kept,
 * per-lane retry iterations, spread retry iterations, rounds with a repeated pick, help probes,
 * then s_memtime cycles: whole attempts, first draws, retries, marking, ring + validation,
 * compaction, claims; then failed validations), then the emit pass's 16.  Only a diagnostics build
 * (-DLDPC_SEQ_STATS=1) collects them; the product build returns LDPC_EUNSUP.
 */
int ldpc_debug_seq_stats(uint64_t *out, int reset);

/*
 * Device diagnostics of the ensemble BEC Monte-Carlo's frontier-peeling decoder
 * (csrc/peel.hip, the message_passing.c:7-82 semantics for the all-zero codeword), collected
 * by the product build on the current device since the last reset: out uint64[3] =
 * {iterations that ran the bitmap-snapshot scan because a frontier list overflowed, trials
 * with at least one such iteration, trials decoded}.  Evidence that the overflow branch ran
 * in a given launch.
 */
int ldpc_debug_peel_stats(uint64_t *out, int reset);

/*
 * Test-only: cap the peeling decoder's frontier-list capacity at F entries (F > 0) so the
 * overflow / scan branch runs deterministically at small n; F <= 0 restores the LDS budget's
 * capacity (5,266 entries at n = 64,800).  Process-wide; results stay bit-exact for any F.
 */
int ldpc_debug_peel_cap(int F);

/* Name of the soft kernel a graph dispatches to (tests / bench); early_stop: 0 fixed count,
 * 1 early stop with posteriors, 2 early stop with hard decisions only (d_post == NULL). */
const char *ldpc_bp_kernel_name(const ldpc_graph *g, int early_stop);

/* ---------------------------------------------------------------------- */
/* Misc                                                                    */
/* ---------------------------------------------------------------------- */
const char *ldpc_last_error(void);
int ldpc_device_count(void);
int ldpc_set_device(int device);
int ldpc_sync(void *stream);

#ifdef __cplusplus
}
#endif
#endif /* LDPC_MI355X_H */
