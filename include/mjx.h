/*
 * mjx.h — C ABI of the MI355X majority-dynamics engine (libmjx.so).
 *
 * Every entry point takes plain device pointers, sizes and a hipStream_t
 * passed as `void*` (NULL = the default stream).  Nothing here allocates,
 * synchronises the device or throws: errors come back as an int status
 * (MJX_OK = 0).  Kernels are hand-written HIP for gfx950.
 *
 * Reference interfaces replaced (paths relative to the thesis repository
 * MarekJankola/Master-Thesis-Optimizing-Initialization-in-Graph-Dynamics-
 * from-Ferromagnetism-to-Opinion-Consensus, "nb" = code/ER_BDCM_entropy.ipynb
 * cited by raw JSON line):
 *
 *   onestep_majority(N, s0)      code/SA_RRG.py:18-20, code/HPR_pytorch_RRG.py:169-171
 *   s_endstate(N, s0, p, c)      code/SA_RRG.py:23-26, code/HPR_pytorch_RRG.py:174-177
 *   onestep_majority (ER)        nb:113-117,  s_endstate (ER) nb:120-123
 *   m(s)                         code/SA_RRG.py:39-40, code/HPR_pytorch_RRG.py:179-180, nb:125-126
 *   E_delta + SA loop body       code/SA_RRG.py:32-37, 63-88
 *   HPr_dp, marginals_comp, new_biases_i   code/HPR_pytorch_RRG.py:137-218
 *   BDCM_ER, Zi_ER, Zij, phi/m_init sums   nb:133-276, 372-392
 *
 * Spin layouts in HBM (bit = 1 means spin +1, bit = 0 means spin -1):
 *
 *   node-packed ("np", one replica): word v>>6, bit v&63 holds node v.
 *       n_words = ceil(n/64).
 *   replica-packed ("rp", R = 64*W replicas): word v*W + (r>>6), bit r&63
 *       holds node v of replica r.  One node's W words are contiguous, so a
 *       neighbour gather moves 8*W contiguous bytes.
 *
 * Adjacency:
 *   ELL (random regular graphs): int32 adj[n*d], row v = neighbours of v
 *       (the reference's `N` array, code/SA_RRG.py:9-16).
 *   CSR (Erdos-Renyi): int64 row_ptr[n+1], int32 col[nnz].
 */
#ifndef MJX_H
#define MJX_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
#define MJX_OK        0
#define MJX_EINVAL    1   /* bad argument (size, degree, null pointer ...) */
#define MJX_EHIP      2   /* a HIP runtime call failed                     */
#define MJX_ERANGE    3   /* size outside what the kernels support         */

/* element types for pack/unpack of +-1 spin arrays */
#define MJX_I8   1
#define MJX_I32  4
#define MJX_I64  8
/* floating-point element types (HPR / BDCM message arrays) */
#define MJX_F32  104
#define MJX_F64  108

int         mjx_abi_version(void);            /* bumps on any signature change */
/* Content hash of the sources (csrc/, include/mjx.h) the library was built
 * from; the Python loader refuses a library whose id differs from its tree. */
const char* mjx_build_id(void);
const char* mjx_strerror(int status);
const char* mjx_last_hip_error(void);         /* text of the last failing HIP call */

/* ---- pack / unpack between +-1 integer arrays and bit layouts ----------- */
/* s: (n,) +-1 of element type `dtype` -> node-packed bits[ceil(n/64)] */
int mjx_pack_np(const void* s, int dtype, int64_t n, uint64_t* bits, void* stream);
int mjx_unpack_np(const uint64_t* bits, int64_t n, void* s, int dtype, void* stream);
/* s: (R, n) row-major +-1 (replica r = row r) -> replica-packed bits[n*W],
 * W = ceil(R/64); padding replicas are written as -1 (bit 0).            */
int mjx_pack_rp(const void* s, int dtype, int64_t n, int64_t R, uint64_t* bits, void* stream);
int mjx_unpack_rp(const uint64_t* bits, int64_t n, int64_t R, void* s, int dtype, void* stream);

/* ---- majority rollout (M1 repeated `steps` times, M2) ------------------ */
/*
 * s_out = onestep^steps(s_in).  For steps >= 2 `tmp` must hold a buffer of
 * the same size as s_in (ping-pong); it may be NULL when steps <= 1.
 * s_in may not alias s_out or tmp.  steps == 0 copies.
 * counts (nullable): per-replica number of +1 spins in s_out, ADDED into
 * counts[R] (uint64; caller zeroes it) — the popcount is fused into the last
 * sweep.  For the np layout R = 1 and counts[0] receives the total.
 */
int mjx_rollout_ell_np(const int32_t* adj, int64_t n, int d,
                       const uint64_t* s_in, uint64_t* s_out, uint64_t* tmp,
                       int steps, unsigned long long* counts, void* stream);
int mjx_rollout_ell_rp(const int32_t* adj, int64_t n, int d, int64_t words,
                       const uint64_t* s_in, uint64_t* s_out, uint64_t* tmp,
                       int steps, unsigned long long* counts, void* stream);
/* mjx_rollout_ell_rp with a graph per replica: R replicas in W = ceil(R/64)
 * words per node; replica r (bit r&63 of word column r>>6) runs on graph
 * rep_graph[r] (device int32[R]) of a stack of graphs, graph g's rows at
 * adj + g*n*d; padding replicas (r >= R) are written as -1 (bit 0).  counts
 * (nullable): [R], added.  The reference's SA draws one graph per replica
 * (code/SA_RRG.py:58-62). */
int mjx_rollout_ell_rp_multi(const int32_t* adj, int64_t n, int d, int64_t R, const int32_t* rep_graph,
                             const uint64_t* s_in, uint64_t* s_out, uint64_t* tmp,
                             int steps, unsigned long long* counts, void* stream);
/* The replica-packed rollout run slice by slice: slice q of S covers word units
 * [q*U/S, (q+1)*U/S) of every node (U = words/2 16-byte units, or words if
 * odd); replicas never interact, so the result is identical for every S.
 * slices = 0 picks S from the state size (mjx_rollout_ell_rp uses that).
 * S must divide U (MJX_EINVAL otherwise). */
int mjx_rollout_ell_rp_sliced(const int32_t* adj, int64_t n, int d, int64_t words,
                              const uint64_t* s_in, uint64_t* s_out, uint64_t* tmp,
                              int steps, int slices, unsigned long long* counts, void* stream);
int mjx_rollout_csr_np(const int64_t* row_ptr, const int32_t* col, int64_t n,
                       const uint64_t* s_in, uint64_t* s_out, uint64_t* tmp,
                       int steps, unsigned long long* counts, void* stream);
int mjx_rollout_csr_rp(const int64_t* row_ptr, const int32_t* col, int64_t n, int64_t words,
                       const uint64_t* s_in, uint64_t* s_out, uint64_t* tmp,
                       int steps, unsigned long long* counts, void* stream);

/* mjx_rollout_csr_rp with a node visiting order (int32 permutation of 0..n-1,
 * nullable): sorted by degree, the two nodes a wavefront holds share one trip
 * count.  Results do not depend on the order. */
int mjx_rollout_csr_rp_ordered(const int64_t* row_ptr, const int32_t* col, const int32_t* order, int64_t n,
                               int64_t words, const uint64_t* s_in, uint64_t* s_out, uint64_t* tmp,
                               int steps, unsigned long long* counts, void* stream);

/* Degree-class ELL: the notebook's own ER layout (nb:113-117 sums
 * s[N_nodes_pos[d]] for the nodes nodes_with_d_positions[d] of each degree
 * class; nb:359-361 builds them), replacing mjx_rollout_csr_rp(_ordered)
 * (`onestep_majority`, nb:113-117; `s_endstate`, nb:120-123).
 * classes: HOST int64 array of nclasses rows {i0, count, D, base}: positions
 * [i0, i0+count) of `order` hold the class's nodes, all of degree D
 * (0 <= D <= 255), and node order[i0+k]'s neighbours are cell[base+k*D ..
 * base+k*D+D); base is a multiple of 4; the counts sum to n.
 * mjx_class_ell_fill writes `cell` from CSR (setup); mjx_rollout_class_rp has
 * the contract of mjx_rollout_csr_rp.  Results do not depend on the layout. */
int mjx_class_ell_fill(const int64_t* row_ptr, const int32_t* col, const int32_t* order,
                       const int64_t* classes, int nclasses, int64_t n, int32_t* cell, void* stream);
int mjx_rollout_class_rp(const int32_t* order, const int32_t* cell, const int64_t* classes, int nclasses,
                         int64_t n, int64_t words, const uint64_t* s_in, uint64_t* s_out, uint64_t* tmp,
                         int steps, unsigned long long* counts, void* stream);
/* Measurement only (no reference counterpart): the class sweep's memory traffic
 * without the majority -- per position its D neighbour rows, its own row where D
 * is even, the rows' XOR written to s_out -- over the same arrays and grid, so
 * the bench can put the sweeps beside the random-row floor of the state. */
int mjx_gather_floor_class(const int32_t* order, const int32_t* cell, const int64_t* classes, int nclasses,
                           int64_t n, int64_t words, const uint64_t* s_in, uint64_t* s_out, void* stream);

/* per-replica count of +1 spins, ADDED into counts (m(s) = (2*count-n)/n) */
int mjx_popcount_np(const uint64_t* bits, int64_t n, unsigned long long* counts, void* stream);
int mjx_popcount_rp(const uint64_t* bits, int64_t n, int64_t words,
                    unsigned long long* counts, void* stream);

/* ---- simulated annealing (code/SA_RRG.py:44-92), R = 64*W replicas ------ */
/*
 * Per-replica state, all device arrays of length R unless noted.  Replica r
 * replays numpy's legacy global MT19937 after np.random.seed(seeds[r]):
 * binomial(1,.5,n) for s0 (code/SA_RRG.py:65), then per step
 * randint(0,n) (:73) and rand() (:76).
 */
typedef struct mjx_sa_state {
    uint32_t* mt;        /* [R*624] MT19937 words, replica-major: mt[r*624 + k] */
    int32_t*  mt_idx;    /* [R] next word index (624 = twist pending)        */
    double*   a;         /* [R] annealing weight a (code/SA_RRG.py:67,80)    */
    double*   b;         /* [R] annealing weight b (:68,81)                  */
    int64_t*  t;         /* [R] proposals made (:82)                         */
    int64_t*  sum_end;   /* [R] sum of s_endstate(s) over nodes (+-1 sum)    */
    int32_t*  done;      /* [R] 0 running, 1 consensus reached, 2 cap hit    */
    int32_t*  prop_i;    /* [R] scratch: proposed node                       */
    int8_t*   prop_s;    /* [R] scratch: spin of the proposed node before the flip */
    double*   prop_u;    /* [R] scratch: accept uniform                      */
    unsigned long long* cnt; /* [R] scratch: +1 count of the rolled-out proposal */
    /* optional per-step trace (NULL to disable); row k = step k of this call */
    int32_t*  tr_i;      /* [nsteps*R] proposed node (-1 if replica done)    */
    int8_t*   tr_acc;    /* [nsteps*R] 1 accepted, 0 rejected, -1 done       */
    int64_t*  tr_sum;    /* [nsteps*R] sum_end after the step               */
    double*   tr_dE;     /* [nsteps*R] delta_H (code/SA_RRG.py:74)          */
    int32_t*  tr_tie;    /* [R] count of |u - exp(-dE)| < 4 ulp near-ties    */
    /* optional proposal tape for mjx_sa_lightcone_steps (NULL / 0 to draw
     * inside the step kernel): the (i, u) of up to tape_cap steps of every
     * replica are drawn ahead by a wave per replica; replica-major: entry
     * (r, k) at r * tape_cap + k, k = step k of the chunk (the library may
     * split the buffer into two halves of tape_cap / 2 rows per replica) */
    int32_t*  tape_i;    /* [tape_cap*R] */
    double*   tape_u;    /* [tape_cap*R] */
    int64_t   tape_cap;
    /* distinct graphs (nullable = every replica on the one graph `adj`):
     * replica r runs on graph rep_graph[r] (device int32[R]) of a stack of
     * graphs with the same n and d, graph g's rows at adj + g*n*d (and at
     * adj_pad + g*n*4 for the padded d = 3 rows).  The reference draws a
     * fresh graph per replica (code/SA_RRG.py:58-62). */
    const int32_t* rep_graph;
    /* light-cone kernel selection, 0 = the library's choice (tests and tuning
     * set them; nothing is read from the environment) */
    int32_t   opt_split;   /* waves per 64-replica word column: 1, 2, 4, ..., 64 */
    int32_t   opt_spec_k;  /* speculative batch width: 8 or 16 */
    uint32_t  opt_flags;   /* MJX_SA_NO_SPEC | MJX_SA_NO_CONE2 | MJX_SA_LDS_* */
    /* nullable: the NON-parity proposal stream.  When set,
     * the tape of mjx_sa_lightcone_steps / _cone_steps / _rec_steps (tape_cap
     * > 0, required) is drawn by Philox-4x32-10 instead of the MT19937 replay:
     * the proposal of step t of replica r is philox4x32_10(counter (t_lo,
     * t_hi, 0, 0), key (k_lo, k_hi)) with k = philox_key[r]: i = the high 64
     * bits of (x0 | x1 << 32) * n, u = (x2 >> 5, x3 >> 6) as numpy's rand().
     * A pure function of (key, t): any chunking, any kernel, same run.  The
     * steps that draw inside the kernel (mjx_sa_steps, mjx_sa_lds_steps)
     * refuse it (MJX_EINVAL). */
    const uint64_t* philox_key;   /* [R] */
    /* library-kept: 1 while the neighbour words of a d = 3, p+c-1 = 2 record
     * array (mjx_sa_rec_*) are current.  mjx_sa_rec_pack writes them; the
     * speculative steps keep them; any other light-cone kernel leaves them
     * stale and sets 0; the next speculative call rebuilds them first.  Start
     * at 0 (a zeroed struct). */
    int32_t   rec_nb;
} mjx_sa_state;

#define MJX_SA_NO_SPEC   1u   /* no speculative batches (k_sa_spec) */
#define MJX_SA_NO_CONE2  2u   /* no one-round-trip step (k_sa_cone2) */
#define MJX_SA_LDS_SERIAL 4u  /* LDS layout: the list-based step (k_sa_lds), not the lane-held one */
#define MJX_SA_LDS_SINGLE 8u  /* LDS layout: one proposal per step (k_sa_lds_fast), not two (k_sa_lds_pair) */
#define MJX_SA_LDS_PAIR  16u  /* LDS layout at p+c-1 = 1: two proposals per step, not eight (k_sa_lds_multi) */
#define MJX_SA_LDS_WAVE  32u  /* LDS layout at p+c-1 >= 2: one wave per replica (k_sa_lds_pair), not the whole
                                 CU (k_sa_lds_wg: opt_split = 4, 8 or 16 waves, one proposal each) */
#define MJX_SA_LDS_CU    64u  /* LDS layout at p+c-1 = 2, 3, d = 3, 4: the whole CU level by level (k_sa_lds_cu:
                                 15 proposals a round, each level's candidates packed over the waves; 8 waves,
                                 16 with opt_split = 16).  The default there where it fits and no other
                                 option is given; opt_split = 4, 8 or 16 alone select k_sa_lds_wg */

/* Seed replica r with seeds[r] (device uint32[R]), draw s0 into the
 * replica-packed spins s[n*W], set a=a0, b=b0, t=0, done=0, and
 * sum_end = sum(s_endstate(s0)) using tmp1/tmp2 ([n*W] each); with
 * st->rep_graph each replica's rollout runs on its own graph. */
int mjx_sa_init(const int32_t* adj, int64_t n, int d, int p, int c, int64_t R,
                const uint32_t* seeds, double a0, double b0,
                uint64_t* s, uint64_t* tmp1, uint64_t* tmp2,
                mjx_sa_state* st, void* stream);

/* As mjx_sa_init, but replica r continues a given MT19937 stream instead of
 * seeding one: mt_in [R*624] words and idx_in [R] next-word indices (device),
 * e.g. the state another replica ended in.  This is how the reference's
 * N_stat replicas share numpy's ONE global stream back to back
 * (code/SA_RRG.py:58-65: replica k+1's s0 draws follow replica k's last rand()). */
int mjx_sa_init_mt(const int32_t* adj, int64_t n, int d, int p, int c, int64_t R,
                   const uint32_t* mt_in, const int32_t* idx_in, double a0, double b0,
                   uint64_t* s, uint64_t* tmp1, uint64_t* tmp2,
                   mjx_sa_state* st, void* stream);

/* Advance every running replica by `nsteps` proposals (code/SA_RRG.py:72-85),
 * full rollout of each proposal.  par_a/par_b: annealing factors (:49-50);
 * a_cap = 4.5*n, b_cap = 5*n (:80-81); t_cap = 2*n**3 (:84). */
int mjx_sa_steps(const int32_t* adj, int64_t n, int d, int p, int c, int64_t R,
                 uint64_t* s, uint64_t* tmp1, uint64_t* tmp2,
                 mjx_sa_state* st, int64_t nsteps,
                 double par_a, double par_b, double a_cap, double b_cap, int64_t t_cap,
                 void* stream);

/* Light-cone SA: the same proposals, accept decisions and
 * outputs as mjx_sa_steps, but each proposal is evaluated only inside the ball
 * of radius p+c-1 around the flipped node, from cached rollout levels.
 * levels: host array of T = p+c-1 device pointers, levels[t-1] = onestep^t(s)
 * (n*W words each), kept consistent by the kernel as flips are accepted.
 * mjx_sa_lightcone_prepare fills them from s (call after mjx_sa_init).
 * Supported: 1 <= T <= 6, d <= 16 and mjx_sa_lightcone_lds(d,p,c) <= 150 KiB
 * (bytes of LDS per 64 replicas; -1 if unsupported).  The step kernel runs
 * several waves per 64-replica word column when the column count is small
 * (st->opt_split overrides the choice).  rep_graph (nullable): as in
 * mjx_sa_state, for the levels of replicas on distinct graphs. */
int64_t mjx_sa_lightcone_lds(int d, int p, int c);
int mjx_sa_lightcone_prepare(const int32_t* adj, int64_t n, int d, int p, int c, int64_t R,
                             const int32_t* rep_graph, const uint64_t* s, uint64_t* const* levels,
                             void* stream);
int mjx_sa_lightcone_steps(const int32_t* adj, int64_t n, int d, int p, int c, int64_t R,
                           uint64_t* s, uint64_t* const* levels, mjx_sa_state* st, int64_t nsteps,
                           double par_a, double par_b, double a_cap, double b_cap, int64_t t_cap,
                           void* stream);

/* Cone layout of the cached levels: the T+1 words (s, onestep(s), ...,
 * onestep^T(s)) of one (node, word column) side by side, padded to
 * LV = mjx_sa_cone_words(p,c) words (2, 4 or 8; -1 if unsupported), word
 * column major: cone[(w*n + v)*LV + t] = level t, word w of node v (n*W*LV
 * words).  A
 * proposal reads several levels of the same nodes; here they share one
 * memory sector.  mjx_sa_cone_pack builds the cone from s and the separate
 * levels (after mjx_sa_lightcone_prepare); mjx_sa_cone_steps is
 * mjx_sa_lightcone_steps on the cone (same proposals, accepts and outputs),
 * mirroring every accepted level-0 flip into s so s stays the configuration;
 * mjx_sa_cone_unpack writes the cone back to s and the separate levels.
 * adj_pad (optional, d = 3): the adjacency with rows padded to 4 int32
 * (n*4, 16-B aligned); with it, p+c-1 = 2 and a proposal tape, every proposal
 * costs one memory round trip (rows fetched down the tape ahead of time). */
int mjx_sa_cone_words(int p, int c);
int mjx_sa_cone_pack(int64_t n, int p, int c, int64_t R, const uint64_t* s,
                     uint64_t* const* levels, uint64_t* cone, void* stream);
int mjx_sa_cone_unpack(int64_t n, int p, int c, int64_t R, const uint64_t* cone,
                       uint64_t* s, uint64_t* const* levels, void* stream);
int mjx_sa_cone_steps(const int32_t* adj, const int32_t* adj_pad, int64_t n, int d, int p, int c, int64_t R,
                      uint64_t* s, uint64_t* cone, mjx_sa_state* st, int64_t nsteps,
                      double par_a, double par_b, double a_cap, double b_cap, int64_t t_cap,
                      void* stream);

/* Record layout: the cone with each (node, word column) sector preceded by the
 * node's adjacency row (int32 x4, zero padded): rec[(w*n + v)*LV + e], words
 * 0..1 = the row, word 2 + t = level t, LV = mjx_sa_rec_words(d,p,c) (4 or 8;
 * -1 if unsupported: d <= 4, p+c-1 <= 5).  The speculative step then fetches a
 * ball node's row and levels in one line.  At d = 3, p+c-1 = 2 the record's
 * spare 28 bytes (the row's pad int, words 5..7) hold its neighbours' level-1
 * bits, 3 per replica (st->rec_nb).  One graph shared by every replica
 * (st->rep_graph must be NULL).  Same proposals, accepts and outputs as every
 * other layout. */
int mjx_sa_rec_words(int d, int p, int c);
/* sizeof(mjx_sa_state) as the library was built (a binding checks its mirror) */
int mjx_sa_state_bytes(void);
int mjx_sa_rec_pack(const int32_t* adj, int64_t n, int d, int p, int c, int64_t R, const uint64_t* s,
                    uint64_t* const* levels, uint64_t* rec, void* stream);
int mjx_sa_rec_unpack(int64_t n, int d, int p, int c, int64_t R, const uint64_t* rec, uint64_t* s,
                      uint64_t* const* levels, void* stream);
int mjx_sa_rec_steps(const int32_t* adj, const int32_t* adj_pad, int64_t n, int d, int p, int c, int64_t R,
                     uint64_t* s, uint64_t* rec, mjx_sa_state* st, int64_t nsteps,
                     double par_a, double par_b, double a_cap, double b_cap, int64_t t_cap,
                     void* stream);

/* LDS-resident light-cone SA (small graphs, the reference's own sizes: n = 1e4,
 * d = 4, code/SA_RRG.py:44-52): a workgroup per replica keeps its graph (uint16
 * rows), the rollout levels onestep^t(s) (t = 0..p+c-1, bit arrays) and its
 * MT19937 state in LDS for the whole call; levels are rebuilt from s at the
 * start of every call, the changed configuration bits XORed back into s and
 * the stream state written back at its end (exactly numpy's position: nothing
 * is drawn ahead).  Same proposals, accepts and outputs as mjx_sa_steps;
 * honours st->rep_graph and the trace pointers; no tape, no level arrays.
 * mjx_sa_lds_bytes: LDS bytes per replica, -1 if (n, d, p, c) does not fit
 * (n <= 65535, d <= 16, 1 <= p+c-1 <= 6, <= 160 KiB). */
int64_t mjx_sa_lds_bytes(int64_t n, int d, int p, int c);
/* LDS bytes per replica of the kernel mjx_sa_lds_steps selects for these
 * kernel options (opt_flags, opt_split), its threads per workgroup in
 * *threads (64, or 64 per wave of the whole-CU kernel); -1 if it does not fit. */
int64_t mjx_sa_lds_plan(int64_t n, int d, int p, int c, uint32_t flags, int split, int* threads);

/* Host-only self-check of the per-device memo tables (CU counts, occupancy,
 * dynamic-LDS opt-ins are kept per device id, not per process): no HIP call,
 * runs without a GPU; 0 = pass, else the number of the failed check. */
int mjx_selftest_devmemo(void);
int mjx_sa_lds_steps(const int32_t* adj, int64_t n, int d, int p, int c, int64_t R, uint64_t* s,
                     mjx_sa_state* st, int64_t nsteps, double par_a, double par_b, double a_cap, double b_cap,
                     int64_t t_cap, void* stream);

/* ---- history-passing reinforcement on d-regular graphs ------------------ */
/*
 * Message arrays use the reference's layout (code/HPR_pytorch_RRG.py:277-285, 46-61):
 * chi[2E][4^T], T = p+c, E = n*d/2; row r < E is G.edges[r] = (u,v) as the
 * message u->v, row r+E is v->u; column of (x_a, x_b) is idx(x_a)*2^T + idx(x_b)
 * with idx(x) = sum_k [x_k = -1] 2^(T-1-k).  Node-major plan arrays, all [n*d]:
 *   nbr[a*d+m]     = m-th neighbour k_m of a
 *   in_row[a*d+m]  = row of the message k_m -> a
 *   out_row[a*d+m] = row of the message a -> k_m   (the reference's N_edges_pos)
 * biases[n][2]: column 0 = bias of spin +1.  dtype MJX_F32 or MJX_F64 for chi,
 * biases, marginals and zwork.
 */
/* HPr_dp (code/HPR_pytorch_RRG.py:183-218): chi_out = damp*chi_new/rowsum +
 * (1-damp)*chi_in, where chi_new carries the reinforced incoming messages
 * (new_biases_chi, :128-133) and the trajectory factor A (:14-39).
 * w_plus / w_minus = exp(-lmbd_in*x_a[0]/n) for x_a[0] = +1 / -1.
 * Supported: 2 <= p+c <= 4, 2 <= d <= 6 (MJX_ERANGE otherwise).
 * chi_in may not alias chi_out. */
int mjx_hpr_update(int dtype, const void* chi_in, void* chi_out, const void* biases,
                   const int32_t* nbr, const int32_t* in_row, const int32_t* out_row,
                   int64_t n, int d, int p, int c, int attr_value,
                   double w_plus, double w_minus, double damp, void* stream);
/* marginals_comp (code/HPR_pytorch_RRG.py:147-167): marg[n][2] (column 0 = +1).
 * zwork: 4E elements of dtype (per-row normalised Z+, Z-). */
int mjx_hpr_marginals(int dtype, const void* chi, const int32_t* out_row, int64_t n, int d,
                      int p, int c, double eps, void* zwork, void* marg, void* stream);
/* new_biases_i (code/HPR_pytorch_RRG.py:137-145) with the uniforms u[n] (float64) the
 * reference draws by torch.rand(n); thresh = 1-(1+t)^(-gamma).  Updates biases in
 * place and writes s[n] = +-1 (int32, nullable). */
int mjx_hpr_new_biases(int dtype, void* biases, const void* marg, const double* u, double thresh,
                       double pie, int64_t n, int32_t* s, void* stream);
/* The same with the comparison u_i < thresh made by the caller: refresh[n] (uint8,
 * nonzero = refresh node i's biases). */
int mjx_hpr_new_biases_mask(int dtype, void* biases, const void* marg, const uint8_t* refresh, double pie,
                            int64_t n, int32_t* s, void* stream);

/* One node step of the HPR main loop in one launch (code/HPR_pytorch_RRG.py:
 * 147-167 node part, 137-145, and the bit packing of s for :352): node
 * marginals from the edge Z sums in zwork (mjx_hpr_marginals_q with marg =
 * NULL computes only those), the bias refresh where refresh[v] (as
 * mjx_hpr_new_biases_mask), s[v] = +-1 and its node-packed bits (as
 * mjx_pack_np).  Replaces mjx_hpr_marginals' node part + new_biases_mask +
 * pack_np; same values. */
int mjx_hpr_node_step(int dtype, const void* zwork, const int32_t* out_row, int64_t n, int d, void* marg,
                      void* biases, const uint8_t* refresh, double pie, int32_t* s, uint64_t* bits, void* stream);
/* The reference's torch.rand(n) per iteration (torch's CPU generator, :142) on the
 * device: state[624] (uint32) and left_next[2] = the CPU engine's `left`, `next`
 * (its get_state() fields); k iterations of n float64 uniforms u = ((y_hi<<32 |
 * y_lo) & (2^53-1)) * 2^-53 from consecutive outputs, compared with thresh[j]
 * (device float64) into mask[j*n + i] (uint8).  state/left_next are left where the
 * CPU generator would be after the same draws.  One workgroup; run it on a
 * stream of its own beside the iterations that consume the masks. */
int mjx_hpr_refresh_masks(uint32_t* state, int32_t* left_next, int64_t n, int k, const double* thresh,
                          uint8_t* mask, void* stream);
/* The same draws by G workgroups at once (MT19937 jump-ahead, csrc/mjx_mtjump.hip):
 * the batch's 2nk words are split into chunks of L words (a multiple of 624), chunk
 * j's workgroup jumps the batch-start state ahead by jL-1 words with the polynomial
 * z^(jL-1) mod P (P = the characteristic polynomial of MT19937's state map).
 * mjx_mt_jump_geometry: L and the number of chunks actually used for (n, k, G);
 * mjx_mt_jump_table_words / mjx_mt_jump_table: the (chunks-1) x 312 uint64 table
 * of those polynomials, computed on the HOST (setup, once per (n, k, G));
 * mjx_hpr_refresh_masks_jump: reads state_in/ln_in (the engine at the batch start),
 * writes state_out/ln_out (after the batch; must not alias the inputs), the masks
 * as mjx_hpr_refresh_masks; `table` is the device copy. */
int mjx_mt_jump_geometry(int64_t n, int k, int G, int64_t* L, int* G_used);
int64_t mjx_mt_jump_table_words(int64_t n, int k, int G);
int mjx_mt_jump_table(int64_t n, int k, int G, uint64_t* table);
int mjx_hpr_refresh_masks_jump(const uint32_t* state_in, const int32_t* ln_in, uint32_t* state_out,
                               int32_t* ln_out, int64_t n, int k, int G, const uint64_t* table,
                               const double* thresh, uint8_t* mask, void* stream);
/* The edge half of marginals_comp (code/HPR_pytorch_RRG.py:150-161) alone:
 * zwork[4E] = per-row normalised (Z+ [2E], Z- [2E]) of every directed row. */
int mjx_hpr_edge_z(int dtype, const void* chi, int64_t E, int p, int c, double eps, void* zwork,
                   void* stream);
/* Node-indexed bias pairs for mjx_hpr_update from the reference's own bias arrays:
 * out[2v+k] = src[idx[v]*stride + k*half], k = 0, 1.  From biases_chi
 * (new_biases_chi, code/HPR_pytorch_RRG.py:128-133): stride = 4^T, half = 4^T/2 and
 * idx[v] = a row whose source node is v; from biases_i: stride 2, half 1. */
int mjx_hpr_node_biases(int dtype, const void* src, const int64_t* idx, int64_t stride, int64_t half,
                        int64_t n, void* out, void* stream);
/* The decay-split layout of the HPR loop state.  HPr_dp writes nothing into the
 * entries of a row whose sender trajectory is invalid (x_s[T-1] != attr_value):
 * they are only damped, chi_t = (1-damp)^t chi_0 (code/HPR_pytorch_RRG.py:215).
 * The loop state keeps each row as quadrants VV | VI | IV | II of (2^(T-1))^2
 * entries (first letter: sender valid/invalid, second: receiver), entry
 * (x_s, x_r) at quad*4^(T-1) + (x_s>>1)*2^(T-1) + (x_r>>1); the IV and II quadrants
 * hold chi_0 undecayed and are read with the scale (1-damp)^t from device
 * memory, so an update reads and writes only the first half of its own rows and
 * the VV and IV quadrants of its incoming rows.
 * mjx_hpr_q_supported: 1 if mjx_hpr_update_q runs this (dtype, d, p, c)
 * (MJX_F32, p+c = 4, 2 <= d <= 4).  mjx_hpr_qlayout: to_q = 1: dst = src
 * (reference layout) permuted; to_q = 0: dst = src (decay-split) in the reference
 * layout with the invalid-sender entries times scale.  mjx_hpr_update_q: HPr_dp on
 * the decay-split layout, *scale_in = chi_in's scale (dtype); chi_out's IV and II
 * quadrants are not written (they must already hold chi_0).  mjx_hpr_marginals_q:
 * marginals_comp of a decay-split chi with scale *scale (marg = NULL: only the
 * edge Z sums into zwork, for mjx_hpr_node_step). */
int mjx_hpr_q_supported(int dtype, int d, int p, int c);
int mjx_hpr_qlayout(int dtype, const void* src, void* dst, int64_t rows, int p, int c, int attr_value, int to_q,
                    double scale, void* stream);
int mjx_hpr_update_q(int dtype, const void* chi_in, void* chi_out, const void* biases, const int32_t* nbr,
                     const int32_t* in_row, const int32_t* out_row, int64_t n, int d, int p, int c,
                     int attr_value, double w_plus, double w_minus, double damp, const void* scale_in,
                     void* stream);
int mjx_hpr_marginals_q(int dtype, const void* chi, const int32_t* out_row, int64_t n, int d, int p, int c,
                        double eps, const void* scale, const void* ii, void* zwork, void* marg, void* stream);
/* ii[4E] (dtype): per edge the four sums of its II x II products (by x_u[0] = +1/-1,
 * by x_v[0] = +1/-1), which never change: computed once from the loop state's
 * chi_0 quadrants; mjx_hpr_marginals_q then skips reading the II quadrants
 * (ii may be NULL: everything is read). */
int mjx_hpr_q_ii(int dtype, const void* chi, int64_t E, int p, int c, void* ii, void* stream);

/* ---- HPR on Erdos-Renyi graphs (the "general (ER)" HPR of code/README.md:1) -
 * HPr_dp with the degree taken per message: rows of degree class D (the
 * message a->b with deg(a) = D+1, rows[m] of them) read their D incoming rows
 * inc[m*D + j] (messages k_j -> a, k_j != b) whose senders are inc_src[m*D + j],
 * with the reinforced messages bias_k(x_k[0]) chi^{k->a} and the trajectory
 * factor of d-1 = D (code/HPR_pytorch_RRG.py:14-39,128-133,183-218); same row,
 * column and bias layouts as mjx_hpr_update.  Jacobi: every class reads chi_in
 * and writes its rows of chi_out.  w_plus/w_minus = exp(-lmbd*x_a[0]/n);
 * 2 <= p+c <= 4, any D <= 255.  A class whose count table (2^(T-1)*(D+1)^T
 * elements per message) does not fit the 160 KiB LDS keeps it in `scratch`:
 * mjx_hpr_er_scratch_bytes(dtype, D, p, c) per message in flight (0: LDS
 * suffices, -1: unsupported); the call then runs ceil(m / (scratch_bytes /
 * that)) launches (MJX_ERANGE if scratch holds not even one table). */
int64_t mjx_hpr_er_scratch_bytes(int dtype, int D, int p, int c);
int mjx_hpr_er_update_class(int dtype, const void* chi_in, void* chi_out, const void* biases,
                            const int32_t* rows, const int32_t* inc, const int32_t* inc_src, int64_t m,
                            int D, int p, int c, int attr_value, double w_plus, double w_minus,
                            double damp, void* scratch, int64_t scratch_bytes, void* stream);
/* node marginals over CSR out-rows (row of i->k for every neighbour k of i):
 * marg[i] = normalised (prod Z+, prod Z-) of zwork from mjx_hpr_edge_z. */
int mjx_hpr_node_marg_csr(int dtype, const void* zwork, int64_t E, const int64_t* out_ptr,
                          const int32_t* out_rows, int64_t n, void* marg, void* stream);

/* ---- one giant graph partitioned by node range -- */
/* One synchronous sweep of the rows [row_lo, row_hi) of a node-packed state.
 * adj holds those rows only: adj[(v - row_lo)*d + k].  s_in / s_out are the
 * full ceil(n/64)-word states (s_in read anywhere, s_out written only in words
 * [row_lo/64, ceil(row_hi/64))).  row_lo must be a multiple of 64 and row_hi a
 * multiple of 64 or n.  counts (nullable): +1 spins among the written nodes,
 * added.  Replaces onestep_majority (code/SA_RRG.py:18-20) on one rank's rows. */
int mjx_sweep_ell_np_range(const int32_t* adj, int64_t n, int d, int64_t row_lo, int64_t row_hi,
                           const uint64_t* s_in, uint64_t* s_out, unsigned long long* counts, void* stream);

/* Source-binned (propagation-blocking) sweep (one replica, huge n; config C5).
 * Same result as mjx_sweep_ell_np_range (code/SA_RRG.py:18-20 on the rows
 * [row_lo, row_hi)); replaces its one-random-cache-line-per-slot gather.  A
 * static plan bins the (row_hi-row_lo)*d (destination, source) slots by source
 * block (1M nodes, staged in LDS) and destination tile (64K nodes, LDS byte
 * counters); a sweep is two streaming kernels (messages, then counts + rule).
 * mjx_binned_plan_shape fills sizes[6] = {src_lo_len (the phase-1 stream),
 * src_hi_len (0: src_hi is unused and may be NULL), off_len (uint16 elements
 * each), index_len (int64 elements), msg_words (uint64 per-sweep message
 * bits), work_bytes (device scratch for mjx_binned_build)}.
 * Limits: n <= 2^31-1, d <= 16; row_lo a multiple of 64, row_hi too unless
 * row_hi == n.  adj holds the rows' ELL entries (global node ids).  */
int mjx_binned_plan_shape(int64_t n, int d, int64_t row_lo, int64_t row_hi, int64_t* sizes);
int mjx_binned_build(const int32_t* adj, int64_t n, int d, int64_t row_lo, int64_t row_hi, uint16_t* src_lo,
                     uint16_t* src_hi, uint16_t* off, long long* index, void* work, int64_t work_bytes, void* stream);
/* apply_form: 0 = the library's choice, 1 = flat tile stream (K <= 960 source
 * blocks, MJX_ERANGE beyond), 2 = per-segment form. */
int mjx_sweep_binned(const uint16_t* src_lo, const uint16_t* src_hi, const uint16_t* off, const long long* index,
                     int64_t n, int d,
                     int64_t row_lo, int64_t row_hi, const uint64_t* s_in, uint64_t* msg, uint64_t* s_out,
                     unsigned long long* counts, int apply_form, void* stream);

/* Device Erdos-Renyi G(n, p) into CSR, replacing
 * nx.erdos_renyi_graph + isolate removal + relabelling of
 * code/ER_BDCM_entropy.ipynb (cell 'ER graph', nb:278-291) with
 * distributional parity: each pair i < j is an edge with probability p
 * (geometric skipping per row, counter-based uniforms of (seed, row, k)).
 * Rows are sorted; the result depends on (n, p, seed) only.  With
 * drop_isolated the degree-0 nodes are removed and the rest relabelled in
 * increasing order (nb:283-291).  row_ptr: int64[n+1] (the first *n_out + 1
 * entries are written), col: int32[col_cap]; *n_out = rows kept, *nnz_out =
 * 2 * edges.  If col_cap < *nnz_out the call returns MJX_ERANGE after setting
 * both (retry with a larger col).  work: mjx_er_work_bytes(n) bytes of device
 * scratch.  Setup call: synchronises `stream`.  n <= 2^31 - 2, 0 <= p < 1.  */
int64_t mjx_er_work_bytes(int64_t n);
int mjx_er_generate(int64_t n, double p, uint64_t seed, int drop_isolated, long long* row_ptr, int32_t* col,
                    int64_t col_cap, int64_t* n_out, int64_t* nnz_out, void* work, int64_t work_bytes, void* stream);

/* ---- device graph generation ----------------------- */
/* Random simple d-regular graph (configuration model through a keyed
 * pseudorandom stub permutation, then deterministic double-edge switches that
 * remove self-loops and multi-edges), replacing nx.random_regular_graph
 * (code/SA_RRG.py:59) with distributional parity.  Writes the ELL rows
 * [row_lo, row_hi) into adj[(row_hi-row_lo)*d]; every rank that calls it with
 * the same (n, d, seed) gets rows of the same graph.  work: device scratch of
 * work_words >= 3 uint64 (defect list; 1 + 2*65536 is ample).  This is a setup
 * call: it synchronises `stream` to run the repair on the host.  n_switches
 * (host, nullable) receives the number of switches made.  d <= 16. */
int mjx_rrg_generate(int64_t n, int d, uint64_t seed, int64_t row_lo, int64_t row_hi, int32_t* adj,
                     uint64_t* work, int64_t work_words, int64_t* n_switches, void* stream);
/* Host-only: partner stub of `stub` in the unrepaired pairing (-1 on bad input). */
int64_t mjx_rrg_partner_host(int64_t n, int d, uint64_t seed, int64_t stub);
/* Checks a full ELL adjacency: counts[0] += self-loops, counts[1] += entries
 * repeated in their row, counts[2] += entries whose reverse multiplicity
 * differs or that are out of range. */
int mjx_graph_check_ell(const int32_t* adj, int64_t n, int d, unsigned long long* counts, void* stream);

/* ---- BDCM on Erdos-Renyi graphs (code/ER_BDCM_entropy.ipynb), float64 ---- */
/*
 * chi[2E][4^T] in the notebook's layout (nb:150-154, 303-314): row r < E is
 * G.edges[r] = (i, j) as the message i -> j, row r + E is j -> i; column of
 * (x_i, x_j) = idx(x_i)*2^T + idx(x_j), idx(x) = sum_t [x_t = +1] 2^(T-1-t).
 * T = p + c <= 4.  An "edge class" is the set of messages a -> b with
 * deg(a) - 1 = D (nb:312-318): rows[m] are their chi rows, inc[m*D + k] the
 * rows of the D incoming messages k -> a (the notebook's N_edges_pos_dm1).
 * Any D <= 255: the count table of an item (2^(T-1)*(D+1)^T doubles) lives in
 * LDS when mjx_bdcm_lds_bytes(D, p, c) <= 160 KiB, else in the caller's
 * `scratch` slab, mjx_bdcm_scratch_bytes(D, p, c) per item in flight (0: LDS
 * suffices, -1: unsupported); the call then runs ceil(m / (scratch_bytes /
 * that)) launches (MJX_ERANGE if the slab holds not even one table).
 */
int64_t mjx_bdcm_lds_bytes(int D, int p, int c);
int64_t mjx_bdcm_scratch_bytes(int D, int p, int c);
/* One class of BDCM_ER (nb:150-196): new rows = damp*normalize(max(chi2, eps))
 * + (1-damp)*old, written to upd[m*4^T] and then committed into chi (the class
 * reads chi before any of its own rows change: Jacobi within a class,
 * Gauss-Seidel across classes when called in ascending D).  damp >= 1 assigns
 * normalize(chi2): with D = 0 that is the leaf reset of nb:404-417.
 * delta_bits (nullable): atomic max of |new - old| as IEEE bits (a NaN wins).
 * gate (nullable): when *gate != 0 on the device the launches do nothing (the
 * stop flag of a captured convergence loop, ctl + 1 below).
 * w_dev (nullable): two doubles {exp(-lmbd), exp(lmbd)} read on the device in
 * place of the lmbd argument, so one captured loop serves every lambda. */
int mjx_bdcm_update_class(double* chi, const int32_t* rows, const int32_t* inc, int64_t m, int D, int p, int c,
                          int attr_value, double lmbd, double damp, double eps, double* upd,
                          unsigned long long* delta_bits, const long long* gate, const double* w_dev, void* scratch,
                          int64_t scratch_bytes, void* stream);
/* The notebook's convergence loop on the device (nb:422-431: while delta > eps,
 * t += 1, stop at T_max), for capture in a hipGraph with one host read per
 * batch.  ctl[4] int64: [0] delta bits of the running sweep (pass ctl as
 * delta_bits), [1] stop flag (pass ctl + 1 as gate), [2] sweeps done t,
 * [3] delta bits of the last completed sweep.  begin: if not stopped, ctl[0] = 0;
 * end: if not stopped, t += 1, ctl[3] = ctl[0], stop when !(delta > eps) or
 * t >= t_max.  Zero ctl before the loop. */
int mjx_bdcm_iter_begin(long long* ctl, void* stream);
int mjx_bdcm_iter_end(long long* ctl, double eps, int64_t t_max, void* stream);
/* Zi_ER for the m nodes of degree D (nb:211-276): zi[nodes[k]] = max(Zi, eps);
 * inc[k*D + j] = row of the message from the j-th neighbour into the node. */
int mjx_bdcm_node_z(const double* chi, const int32_t* nodes, const int32_t* inc, int64_t m, int D, int p, int c,
                    int attr_value, double lmbd, double eps, double* zi, void* scratch, int64_t scratch_bytes,
                    void* stream);
/* Zij (nb:200-209) and the per-edge term of avg_m_init (nb:379-392);
 * edges[2E] = G.edges (u, v) pairs, deg[n] node degrees; m_term nullable. */
int mjx_bdcm_edge_obs(const double* chi, const int32_t* edges, const int32_t* deg, int64_t E, int p, int c,
                      int attr_value, double eps, double* zij, double* m_term, void* stream);
/* out[0] = sum_i x[i] (take_log: sum_i log x[i]), deterministic order;
 * work: 256 doubles of device scratch. */
int mjx_sum_f64(const double* x, int64_t n, int take_log, double* work, double* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* MJX_H */
