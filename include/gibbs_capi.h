/*
 * gibbs_capi.h -- C-ABI of libgibbs_hip.so, the MI355X-native Gibbs hot path.
 *
 * Plain pointers and sizes only.  All array pointers passed to gs_* compute
 * calls are DEVICE pointers (caller-owned, e.g. torch tensor.data_ptr());
 * gs_model_desc carries HOST pointers that are copied once at plan creation.
 * Every compute call is asynchronous on the given hipStream_t (passed as
 * void*, NULL = default stream) and returns 0 on success, <0 on error with a
 * message in gs_last_error().  A plan is bound to the device that was current
 * when it was created; it is not thread-safe.  No call allocates, copies
 * host<->device or synchronises, so every step is capturable in a hipGraph.
 *
 * Reference interfaces replaced (Gabriel-Ducrocq/GibbsSampler, file:line):
 *   gs_var_expand            utils.generate_var_cl             utils.py:114-147,
 *                            variance_expension.generate_var_cl_cython  variance_expension.pyx:8-33
 *   gs_real_to_complex       utils.real_to_complex             utils.py:49-60, variance_expension.pyx:84-100
 *   gs_complex_to_real       utils.complex_to_real             utils.py:63-76, variance_expension.pyx:65-81
 *   gs_remove_monopole_dipole  remove_monopole_dipole_contributions  variance_expension.pyx:103-111
 *   gs_alm2cl                hp.alm2cl on real-layout a_lm     CenteredGibbs.py:30,61
 *   gs_unfold_bins           utils.unfold_bins                 utils.py:150-162
 *   gs_block_params          per-l Sigma/Cholesky of the CR    CenteredGibbs.py:324-337 (centered),
 *                            NonCenteredGibbs.py:141-151 (non-centered); TEB 3x3 semantics of the
 *                            cp38 helpers compute_inverse_and_cholesky / compute_sigma_and_chol
 *   gs_cr_sweep              the Gaussian CR draw + alm2cl/sufficient-statistic reduction
 *                            CenteredGibbs.py:340-353, NonCenteredGibbs.py:160-176
 *   gs_cls_draw              PolarizedCenteredClsSampler.sample CenteredGibbs.py:54-93 (+ TEB inverse-Wishart)
 *   gs_nc_mh                 PolarizationNonCenteredClsSampler.sample NonCenteredGibbs.py:292-445 (all_sph)
 *   gs_stats_to_noncentered  ASIS non-centering s_nc = C^-1/2 s  ASIS.py:185-189
 *   gs_step_centered / gs_step_noncentered / gs_step_asis
 *                            one iteration of GibbsSampler.run_polarization GibbsSampler.py:142-173,
 *                            NonCenteredGibbs.run_polarization NonCenteredGibbs.py:546-560,
 *                            ASIS.run_polarization ASIS.py:158-206
 *
 * Layouts (fp64):
 *   real a_lm layout, NR = (L+1)^2 per field (utils.py:49-76); alm arrays are
 *   [nchains][nfields][NR]; data d_alm is [nfields][NR] (shared by chains).
 *   binned spectra: [nchains][nspec][maxbins] (maxbins = max over spectra).
 *   statistics: [nchains][nstat][L+1], see GS_NSTAT_* below.
 *   fields: nfields=1 (T), 2 (E,B), 3 (T,E,B); spectra: [TT] / [EE,BB] /
 *   [TT,EE,BB,TE].
 *
 * RNG: replay mode when the variate pointer is non-NULL (host-drawn numpy
 * variates in the reference's draw order); native mode otherwise
 * (Philox4x32-10 keyed by (seed, global chain id), counter = (element,
 * field, tag|substep, iteration); independent of launch geometry).
 */
#ifndef GIBBS_CAPI_H
#define GIBBS_CAPI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GS_ABI_VERSION 1

#define GS_MODE_CENTERED 0
#define GS_MODE_NONCENTERED 1

#define GS_QUIRK_ASIS_RECENTRE_CENTERED 1   /* ASIS.py:203 re-centres the centered map */

/* number of per-l statistics per chain, by nfields:
 *  1: [ssTT, dTsT]
 *  2: [ssEE, ssBB, dEsE, dBsB]
 *  3: [ssTT, ssEE, ssBB, ssTE, dTsT, dEsT, dEsE, dBsB]
 * ss = sum over the slots of l of s_X s_Y ; dXsY = sum of d_X s_Y. */
#define GS_NSTAT_1 2
#define GS_NSTAT_2 4
#define GS_NSTAT_3 8
#define GS_NPARAM 10   /* doubles per (chain, l) in a block-parameter table */

typedef struct gs_plan gs_plan;

typedef struct gs_model_desc {
    int lmax;                 /* L                                           */
    int nside;                /* HEALPix N_side (Npix = 12 N_side^2)          */
    int nfields;              /* 1, 2 or 3                                    */
    int nchains;              /* chains batched in this plan                  */
    int chain0;               /* global id of the plan's first chain (RNG key) */
    int quirks;               /* GS_QUIRK_* bit set                           */
    int n_iter_metropolis;    /* MH attempts per block (NonCenteredGibbs.py:427) */
    const double* bl;         /* host [L+1] beam b_l                          */
    const double* noise_var;  /* host [nfields] per-pixel noise variance      */
    const int* bins[4];       /* host bin edges per spectrum                  */
    int nbin_edges[4];        /* number of edges (= nbins + 1)                */
    const int* blocks[4];     /* host MH block edges per spectrum (nullable)  */
    int nblock_edges[4];
    const double* prop_var[4];/* host [nbins-2] MH proposal variances (nullable) */
} gs_model_desc;

int gs_abi_version(void);
const char* gs_last_error(void);

/* Library options: named settings read when a plan, SHT or masked context is
 * created (the library reads no environment variables).  Speed-only shape
 * selectors (every value gives the same bits) and the variant switches the
 * bit-identity tests compare, plus the f2 / table workspace budgets:
 *   GS_SWEEP_TW          1 | 2 | 4  CR-sweep workgroup shape (tiles x chunks;
 *                                   2 suits --skymap store, 1 the default)
 *   GS_SWEEP_THROUGHPUT  1          few-chain plans use the throughput form
 *   GS_MH_SPLIT          0 | 1      NC MH in one / two workgroups per chain
 *   GS_CLS_PRE, GS_CLS_PRE_MANY  0 | 1  C_l-draw variates inside the sweep
 *   GS_F2_GROUP_BYTES, GS_F2_BATCH_BYTES  f2 workspace budgets (bytes)
 *   GS_SHT_LDS_FFT_MAX, GS_SHT_SEG, GS_SHT_SYN, GS_SHT_ANA, GS_SHT_MERGE_RINGS,
 *   GS_SHT_CONST_RINGS, GS_SHT_BLOCKS_MFMA, GS_SHT_BLK_STAGE, GS_SHT_FUSED_AUX,
 *   GS_SHT_MFMA_MAX_GB, GS_SHT_RING_TW2  SHT launch shapes / paths (gs_sht.hip
 *                        documents each)
 * gs_option_set(name, NULL) unsets; an unknown name is an error. */
int gs_option_set(const char* name, const char* value);
const char* gs_option_get(const char* name);   /* NULL when unset or unknown */

int gs_plan_create(const gs_model_desc* desc, gs_plan** out);
int gs_plan_destroy(gs_plan* plan);
/* query sizes of the plan's layouts */
int gs_plan_info(const gs_plan* plan, int* maxbins, int* nstat, int* nblocks_total, int* nspec);
/* tiling of the CR sweep: tasks per chain, m-rows per task */
int gs_plan_sweep_info(const gs_plan* plan, int* ntask, int* rows_per_task);

/* ---- stand-alone layout / expansion helpers (no plan needed) ---------------- */
int gs_var_expand(int lmax, int n, const double* dl, double* var, void* stream);
int gs_real_to_complex(int lmax, int n, const double* re, double* cplx_interleaved, void* stream);
int gs_complex_to_real(int lmax, int n, const double* cplx_interleaved, double* re, void* stream);
int gs_remove_monopole_dipole(int lmax, int n, double* alm, void* stream);
int gs_alm2cl(int lmax, int n, const double* x, const double* y, double* cl, void* stream);
int gs_unfold_bins(int n, const double* binned, const int* bins, int nbins, double* out, void* stream);

/* ---- plan-level hot-path stages ------------------------------------------- */
/* per-(chain, l) (M, Cholesky) table of the CR: s = M d + Lchol z */
int gs_block_params(gs_plan* plan, int mode, const double* dl_binned, double* params, void* stream);
/* fused CR draw + statistics: writes s (nullable => not stored) and stats */
int gs_cr_sweep(gs_plan* plan, const double* d_alm, const double* params, const double* z_replay,
                uint64_t seed, uint32_t iteration, uint32_t substep,
                double* s_out, double* stats, void* stream);
/* statistics (alm2cl auto/cross + data correlations) of a given s
 * [nchains][nfields][NR] -- hp.alm2cl of CenteredGibbs.py:30,61 */
int gs_sweep_stats(gs_plan* plan, const double* d_alm, const double* s, double* stats, void* stream);
/* centered C_l draw (inverse-Gamma; TEB: inverse-Wishart TT/EE/TE) */
int gs_cls_draw(gs_plan* plan, const double* stats, const double* invgamma_replay,
                uint64_t seed, uint32_t iteration, double* dl_binned_out, void* stream);
/* non-centered Metropolis-within-Gibbs over blocks (in/out dl_binned) */
/* proposals of the NC Metropolis step (NonCenteredGibbs.py:292-330) into caller
 * buffers [nchains][nspec][maxbins] (prop, log proposal ratio) and, when
 * u_acc_out != NULL, the native accept uniforms [nchains][nacc]; used by the
 * pixel-domain (masked) MH whose block loop needs a full SHT per block. */
int gs_mh_propose(gs_plan* plan, const double* dl, const double* u_prop, uint64_t seed, uint32_t iteration,
                  double* prop_out, double* logr_out, double* u_acc_out, void* stream);
int gs_nc_mh(gs_plan* plan, const double* stats, double* dl_binned,
             const double* u_prop_replay, const double* u_accept_replay,
             uint64_t seed, uint32_t iteration, int32_t* accept_out, void* stream);
/* stats of s_nc = A(C)^+ s with A = chol(C(dl_binned)) (ASIS non-centering) */
int gs_stats_to_noncentered(gs_plan* plan, const double* dl_binned, double* stats, void* stream);
/* s <- T_l s for T_l = A(C(dl_new)) [A(C(dl_old))^+ unless dl_old NULL] */
int gs_recentre(gs_plan* plan, const double* dl_new, const double* dl_old, double* s, void* stream);

/* ---- fused iterations ------------------------------------------------------ */
int gs_step_centered(gs_plan* plan, const double* d_alm, double* dl_binned, double* s_out,
                     const double* z_replay, const double* invgamma_replay,
                     uint64_t seed, uint32_t iteration, void* stream);
/* native RNG, device iteration counter on (graph-captured steps): gs_step_centered
 * with the D_l trace record (trace nullable: [capacity][nchains][nspec][maxbins],
 * slot (iteration - 1) % capacity) and the counter advance in the C_l-draw launch */
int gs_step_centered_fused(gs_plan* plan, const double* d_alm, double* dl_binned, double* s_out,
                           uint64_t seed, uint32_t iteration, double* trace, int capacity, void* stream);
/* the same for gs_step_asis (native): trace record and counter advance in the MH launch */
int gs_step_asis_fused(gs_plan* plan, const double* d_alm, double* dl_binned, double* s_out,
                       uint64_t seed, uint32_t iteration, int32_t* accept_out, double* dl_tmp_out, int recentre,
                       double* trace, int capacity, void* stream);
int gs_step_noncentered(gs_plan* plan, const double* d_alm, double* dl_binned, double* s_out,
                        const double* z_replay, const double* u_prop_replay, const double* u_accept_replay,
                        uint64_t seed, uint32_t iteration, int32_t* accept_out, void* stream);
/* the three stages of gs_step_noncentered, for callers that schedule them:
 *   gs_nc_prologue  the MH proposals (and native accept uniforms) of dl
 *                   (NonCenteredGibbs.py:292-330) and, for plans of more than 4
 *                   chains, the NC block parameters of dl (:134-176)
 *   gs_nc_sweep     the CR draw + sufficient statistics; plans of <= 4 chains
 *                   compute the NC operator of dl per l inside the sweep
 *   gs_nc_decide    the Metropolis-within-Gibbs decisions (NonCenteredGibbs.py:401-445)
 * Native RNG, plans of more than 4 chains: the prologue launches the block
 * parameters only and the proposals / accept uniforms are drawn by the launch
 * that reduces the statistics (gs_nc_sweep with finish = 1, or gs_nc_finish);
 * the decide calls fail if that launch has not run since the prologue.  With
 * GS_NC_MH_PARAMS=1 at plan creation, inside a captured multi-step graph
 * (gs_graph_step offset > 0) the previous step's gs_nc_decide_fused wrote this
 * step's parameters and the prologue launches nothing.  GS_NC_PRO_DEFER=0: all
 * in the prologue (the same values either way). */
int gs_nc_prologue(gs_plan* plan, const double* dl_binned, const double* u_prop_replay, uint64_t seed,
                   uint32_t iteration, void* stream);
int gs_nc_sweep(gs_plan* plan, const double* d_alm, const double* dl_binned, double* s_out, const double* z_replay,
                uint64_t seed, uint32_t iteration, int finish, void* stream);
/* finish = 0 leaves the statistics as per-task partials; gs_nc_finish reduces them
 * (fixed order) -- lets a caller bracket the sweep kernel alone with timing events */
int gs_nc_finish(gs_plan* plan, void* stream);
int gs_nc_decide(gs_plan* plan, double* dl_binned, const double* u_accept_replay, uint64_t seed, uint32_t iteration,
                 int32_t* accept_out, void* stream);
/* gs_nc_decide with the step's bookkeeping fused into the same launch (native
 * RNG, for graph-captured steps): after the decisions each chain's workgroup
 * records its D_l in trace (nullable; trace[(it-1) % capacity]) and, with the
 * device counter on, the last workgroup advances the counter (ticket; every
 * workgroup read it at its start). */
int gs_nc_decide_fused(gs_plan* plan, double* dl_binned, uint64_t seed, uint32_t iteration, int32_t* accept_out,
                       double* trace, int capacity, void* stream);
/* dl_tmp_out: nullable, receives the centered draw; recentre: 0 lazy (s_out keeps the
 * centered CR draw), 1 materialise the re-centred map in s_out */
int gs_step_asis(gs_plan* plan, const double* d_alm, double* dl_binned, double* s_out,
                 const double* z_replay, const double* invgamma_replay,
                 const double* u_prop_replay, const double* u_accept_replay,
                 uint64_t seed, uint32_t iteration, int32_t* accept_out, double* dl_tmp_out,
                 int recentre, void* stream);

/* hipGraph support: with the device counter enabled every RNG-consuming
 * kernel reads the iteration as a device base word plus the step's offset
 * (the host iteration argument is ignored), so a captured graph replays as
 * the next iterations.  gs_graph_step(offset, advance) sets the offset of the
 * steps launched next (0 after gs_iteration_counter) and how far the fused
 * entry points' last launch advances the base (1 after gs_iteration_counter:
 * one captured step per replay; a graph of K steps passes offsets 0..K-1 and
 * advance K on its last step, 0 on the others -- one ticket per replay).
 * gs_advance_iteration increments the base by one from the stream. */
int gs_iteration_counter(gs_plan* plan, int enable, uint32_t start);
int gs_graph_step(gs_plan* plan, uint32_t offset, uint32_t advance);
int gs_advance_iteration(gs_plan* plan, void* stream);
/* trace[(it-1) % capacity][nchains][nspec][maxbins] <- dl_binned (history of GibbsSampler.py:172-173) */
int gs_record_trace(gs_plan* plan, const double* dl_binned, double* trace, int capacity, uint32_t iteration,
                    void* stream);

/* device-side timing of the dominant kernel: with enable = 1 every later CR-sweep
 * launch is bracketed by hipEvents on its stream (also while the stream is
 * captured into a hipGraph: external event-record nodes, timed at each replay);
 * enable = 2 / 3 pause / resume (launches in between are not bracketed);
 * enable = 0 returns the summed duration and the number of launches timed */
int gs_sweep_timing(gs_plan* plan, int enable, double* total_ms, int* count);

/* ---- HEALPix RING spherical-harmonic transforms (gs_sht.hip) ------------
 * Replace healpy's hp.alm2map / hp.map2alm as called by the masked CR
 * variants: CenteredGibbs.py:204,298,505,513,698,717,751,773,791,812,
 * NonCenteredGibbs.py:155,350, utils.adjoint_synthesis_hp utils.py:79-111.
 * ncomp: 1 = T (spin 0), 2 = (E,B) <-> (Q,U) (spin 2), 3 = (T,E,B) <-> (T,Q,U).
 * alm layout: GS_ALM_REAL (real m-major, (L+1)^2 doubles per component,
 * utils.py:49-76) or GS_ALM_COMPLEX (healpy order, (L+1)(L+2)/2 complex
 * interleaved per component).  maps: [ncomp][12 nside^2] RING order.
 * map2alm = (4 pi / Npix) x adjoint of alm2map (healpy, uniform weights);
 * niter adds healpy's Jacobi refinements a += map2alm(m - alm2map(a)).
 * One SHT plan serves one stream at a time (it owns the ring-phase workspace). */
#define GS_ALM_REAL 0
#define GS_ALM_COMPLEX 1
typedef struct gs_sht gs_sht;
int gs_sht_create(int nside, int lmax, gs_sht** out);
int gs_sht_destroy(gs_sht* sht);
int gs_sht_info(const gs_sht* sht, int* nside, int* lmax, long long* npix, long long* device_bytes);
int gs_sht_alm2map(gs_sht* sht, int ncomp, int layout, const double* alm, double* maps, void* stream);
int gs_sht_map2alm(gs_sht* sht, int ncomp, int layout, const double* maps, double* alm, int niter, void* stream);
/* Fused forms of the masked CR's transform pairs (real layout, iter 0):
 *   alm2map_beamed   = hp.alm2map(almxfl(alm, b_l))       (CenteredGibbs.py:698-699,752-753)
 *   map2alm_weighted = hp.map2alm(weights * maps, iter=0) (CenteredGibbs.py:298-299,510-513)
 * bit-identical to a separate per-l / per-pixel multiply followed by the plain
 * transform (the product is rounded once, on the transform's input load). */
int gs_sht_alm2map_beamed(gs_sht* sht, int ncomp, const double* alm_real, const double* bl, double* maps, void* stream);
int gs_sht_map2alm_weighted(gs_sht* sht, int ncomp, const double* maps, const double* weights, double* alm_real,
                            void* stream);
/* Batches of maps (one per chain; the reference runs its chains as separate
 * SLURM tasks, job-script.sh:6-8, each calling hp.alm2map / hp.map2alm):
 * alm [nmap][ncomp][n], maps [nmap][ncomp][Npix] contiguous; one launch per
 * stage serves every map (small maps fill the GPU), and map b of a batch is
 * bit-identical to the same map transformed alone.  bl (nullable, real layout):
 * per-l beam on the synthesis input (hp.alm2map(almxfl(alm, b_l))); weights
 * (nullable; real layout, niter 0): [ncomp][Npix] shared by the batch, the
 * analysis of weights * maps (hp.map2alm(N^-1 m)).  gs_sht_reserve sizes the
 * plan's per-map workspace for nmap maps ahead of a graph capture (a larger
 * batch inside a capture is an error). */
int gs_sht_reserve(gs_sht* sht, int nmap, void* stream);
/* on = 1: the plan's Legendre stage runs on the fp64 matrix cores from a
 * plan-time table of lambda (8 B per (l, m, ring pair): 0.54 GB at N_side 256,
 * 4.3 GB at N_side 512; budget GS_SHT_MFMA_MAX_GB, default 16; the spin-2 F1 /
 * F2 are formed in the kernels) -- a dense contraction per m whose inner
 * dimension every map of a batch shares.
 * Every transform of the plan then uses it (a map's result does not depend on
 * the batch size); on = 0 returns to the on-the-fly recurrence kernels.
 * Small maps only (plans without split-ring FFTs).  _info: state, table bytes. */
int gs_sht_set_mfma(gs_sht* sht, int on);
int gs_sht_mfma_info(const gs_sht* sht, int* on, long long* table_bytes);
int gs_sht_alm2map_batch(gs_sht* sht, int nmap, int ncomp, int layout, const double* alm, const double* bl,
                         double* maps, void* stream);
/* the masked PCG operator's transform pair in one call: alm_out =
 * map2alm(weights x alm2map(bl x alm_in)), real layout, niter 0 (the
 * reference's hp.map2alm(N^-1 hp.alm2map(almxfl(s, b_l))) of its PCG fwd_op,
 * CenteredGibbs.py:448-491).  On the matrix-core table path with the
 * multi-component ring stage the per-ring synthesis, weighting and analysis run
 * in one workgroup and the maps never reach HBM (bit-identical to the two
 * calls); otherwise the two calls through maps_scratch ([nmap][ncomp][Npix],
 * may be NULL only on the fused path). */
int gs_sht_apply_weighted_batch(gs_sht* sht, int nmap, int ncomp, const double* alm_in, const double* bl,
                                const double* weights, double* maps_scratch, double* alm_out, void* stream);
int gs_sht_map2alm_batch(gs_sht* sht, int nmap, int ncomp, int layout, const double* maps, const double* weights,
                         double* alm, int niter, void* stream);

/* ---- masked (pixel-domain) constrained realisation (gs_masked.hip) -------
 * Replaces PolarizedCenteredConstrainedRealization's masked samplers:
 *   GS_MCR_AUX        sample_gibbs_change_variable  CenteredGibbs.py:676-729
 *   GS_MCR_OVERRELAX  overrelaxation_sampler        CenteredGibbs.py:733-825
 *   GS_MCR_MALA       sample_mala                   CenteredGibbs.py:560-603 (EB only)
 *   GS_MCR_AUX_MALA   the ula composition of sample CenteredGibbs.py:832-836
 * A context runs a batch of B = desc.nchains chains (0 -> 1) on one data set:
 * the reference's independent chains (its SLURM array, job-script.sh:6-8) as
 * one batch whose transforms are batched SHTs; `chain` arguments are the global
 * id of the batch's first chain (chain b has id chain + b), and chain b's
 * results equal a one-chain context's for id chain + b bit for bit when both
 * contexts run the same Legendre stage (desc.sht_mode resolved to the same
 * path: "auto" = 0 picks the matrix-core tables from 4 chains on small maps and
 * the recurrence otherwise, so pass 1 or 2 explicitly to compare a batch with a
 * one-chain run; the two paths agree to ~1e-12 relative).
 * maps / inv_noise (create): DEVICE [3][Npix] rows T, Q, U (inv_noise
 * mask-multiplied, CenteredGibbs.py:266-274; the T row is read only for
 * nfields = 3), shared by the batch.  Every per-chain argument is [B][...]
 * contiguous: dl DEVICE unbinned D_l [B][nspec][L+1]; s [B][F][(L+1)^2] real
 * layout, updated in place; v [B][F][Npix] the auxiliary map (needed across
 * calls only by GS_MCR_OVERRELAX; may be NULL).  Replay variates (NULL =
 * native Philox streams), per chain: zv [B][n][F][Npix] pixel normals, zs
 * [B][n][F][NR] slot normals in the reference's draw order (AUX: per inner
 * iteration v then s; OVERRELAX: initial v, then per iteration s, v, s; MALA:
 * zm [B][F][NR], um [B]).  accept (device int32 [B], optional): 1 for the
 * auxiliary samplers, the MALA decisions otherwise; log_ratio (device double
 * [B], optional). */
#define GS_MCR_AUX 0
#define GS_MCR_OVERRELAX 1
#define GS_MCR_MALA 2
#define GS_MCR_AUX_MALA 3
typedef struct gs_masked gs_masked;
typedef struct gs_masked_desc {
    int lmax, nside, nfields;      /* nfields 1 (T), 2 (E,B) or 3 (T,E,B)         */
    const double* bl;              /* HOST [L+1] beam                             */
    int n_gibbs;                   /* inner iterations (CenteredGibbs.py:250)     */
    double alpha;                  /* over-relaxation, -0.995 (CenteredGibbs.py:244) */
    double tau;                    /* MALA step, 0.02 (CenteredGibbs.py:294)      */
    double noise_pol0;             /* noise_pol[0] of the MALA sigma (571-572)    */
    double mu_eps;                 /* mu = max(N^-1) + mu_eps; 0 -> 1e-14 (pol,   */
                                   /* CenteredGibbs.py:276); TT: 1e-7              */
                                   /* (ConstrainedRealization.py:44)              */
    int adj_iter;                  /* map2alm iterations of the data term          */
                                   /* b A^T N^-1 d and of the aux s|v analysis:    */
                                   /* 0 (pol: iter=0) or 3 (TT: adjoint_synthesis_hp */
                                   /* and healpy's default, CenteredGibbs.py:208)  */
    int nchains;                   /* chains of the batch (0 or 1: one chain)     */
    int sht_mode;                  /* Legendre stage: 0 auto (the matrix-core    */
                                   /* table path for batches of >= 4 chains when  */
                                   /* its table fits), 1 on-the-fly recurrence,   */
                                   /* 2 the matrix-core table path                */
} gs_masked_desc;
int gs_masked_create(const gs_masked_desc* desc, const double* maps, const double* inv_noise, gs_masked** out);
int gs_masked_destroy(gs_masked* ctx);
/* Diagnostic (no reference counterpart): the context's N^-1 ring-pair classes,
 * computed once at create -- counts[0] pairs without weight, counts[1] pairs
 * with a ring whose weights vary, counts[2] pairs whose weights are one number
 * per ring (isotropic noise on rings the mask leaves whole: the PCG operator's
 * ring stage and the f2 Gram pass take their constant-ring forms there). */
int gs_masked_ring_classes(const gs_masked* ctx, int* counts /* HOST [3] */);
int gs_masked_info(const gs_masked* ctx, double* mu3 /* HOST [3] */, double* second_part_grad /* DEVICE [F][NR] */);
int gs_masked_nchains(const gs_masked* ctx);   /* chains of the batch; -1 for a null context */
int gs_masked_sht_tables(const gs_masked* ctx); /* 1: the matrix-core table path is on, 0: off */
int gs_masked_gradient(gs_masked* ctx, const double* dl, const double* s, double* grad, double* pix, void* stream);
/* f4: temperature full-sky CR from pixel data (nfields = 1 context):
 * centered CenteredConstrainedRealization.sample_no_mask (CenteredGibbs.py:108-132)
 * or non-centered NonCenteredConstrainedRealization.sample_no_mask
 * (NonCenteredGibbs.py:22-38); zv [Npix] / zs [NR] replay normals (reference
 * order: zs then zv) or NULL for the native streams; s_out [NR]. */
int gs_masked_tt_fullsky(gs_masked* ctx, int noncentered, const double* dl, const double* zv, const double* zs,
                         uint64_t seed, uint32_t iteration, int chain, double* s_out, void* stream);
int gs_masked_cr(gs_masked* ctx, int kind, const double* dl, double* s, double* v, const double* zv, const double* zs,
                 const double* zm, const double* um, uint64_t seed, uint32_t iteration, int chain, int32_t* accept,
                 double* log_ratio, void* stream);
/* f1: the PCG CR (sample_mask, CenteredGibbs.py:448-491).  rhs = b A^T N^-1 d
 * + b adjoint_synthesis_hp(sqrt(N^-1) z_pix) (map2alm iter=3, utils.py:79-111)
 * + C^-1/2 z_slot; solve (C^+ + b A^T N^-1 A b) x = rhs by preconditioned CG
 * (per-l preconditioner (C^+ + b^2 nbar/w)^-1) until |r| <= tol |rhs|.
 * zv [F][Npix], zs [F][NR]: replay normals (reference order z_Q, z_U, z_E,
 * z_B) or NULL for the native streams.  The CG recurrence's scalars stay on
 * the device; the host launches batches of iterations sized from the residual's
 * decay and synchronises once per batch (no host round trip per iteration).
 * Batched contexts solve every chain's system at once (per-chain scalars and
 * convergence; rhs / x [B][F][NR]); iters / rel_residual are HOST [B].
 * gs_masked_pcg_info: host synchronisations of the last solve; _info2 also the
 * CG iterations launched (>= every chain's count: a converged chain's kernels
 * return at once, its transforms still run until the batch's last chain
 * converges). */
int gs_masked_pcg_rhs(gs_masked* ctx, const double* dl, const double* zv, const double* zs, uint64_t seed,
                      uint32_t iteration, int chain, double* rhs, void* stream);
int gs_masked_pcg_solve(gs_masked* ctx, const double* dl, const double* rhs, double* x, int x_is_guess, double tol,
                        int maxiter, int* iters, double* rel_residual, void* stream);
int gs_masked_pcg_info(const gs_masked* ctx, int* host_syncs);
int gs_masked_pcg_info2(const gs_masked* ctx, int* host_syncs, int* launched);
/* The last solve's transformed chain-iterations: the sum over its launched CG
 * iterations of the chains still unconverged at the last state read (the batch
 * transforms only those; launched x B without that compaction). */
int gs_masked_pcg_work(const gs_masked* ctx, long long* chain_iterations /* HOST */);
/* out = Q x, the PCG system operator (C^+ + b A^T N^-1 A b) applied to x
 * (qcinv opfilt_pp fwd_op, CenteredGibbs.py:631,655). */
int gs_masked_pcg_apply(gs_masked* ctx, const double* dl, const double* x, double* out, void* stream);
/* RJPO accept step (sample_mask_rj, CenteredGibbs.py:606-674): x is the PCG
 * solution of Q x = rhs started from -s (gs_masked_pcg_solve with x = -s as the
 * guess, :645-650); log_ratio = -sum (rhs - Q x) . (s - x) (:657-669), accept
 * when log u < log_ratio (:670) and then s <- x.  um: device [1] replay uniform
 * or NULL for the native stream (Philox(0, 0, TAG_RJ_U, iteration)); accept,
 * log_ratio: device int32 [1] / double [1] or NULL.  Nothing is read back. */
int gs_masked_rj_accept(gs_masked* ctx, const double* dl, const double* rhs, const double* x, double* s,
                        const double* um, uint64_t seed, uint32_t iteration, int chain, int32_t* accept,
                        double* log_ratio, void* stream);
/* f2: pixel-domain non-centered likelihood (NonCenteredGibbs.py:333-355):
 * lik = -1/2 sum_pix N^-1 (d - A b C^1/2(D) s_nc)^2 (device double).
 * gs_masked_center: out = C^1/2 in (dir = +1) or C^+1/2 in (dir = -1) per slot
 * (EB sqrt(var) / sqrt(inv_var), NonCenteredGibbs.py:236-237; TEB chol(C)). */
int gs_masked_center(gs_masked* ctx, const double* dl, int dir, const double* in, double* out, void* stream);
int gs_masked_nc_loglik(gs_masked* ctx, const double* dl, const double* s_nc, double* lik, void* stream);
/* f2: one Metropolis sweep of the pixel-domain non-centered likelihood over K
 * blocks (PolarizationNonCenteredClsSampler.sample / NonCenteredClsSampler.sample
 * with all_sph=False, NonCenteredGibbs.py:401-445 with :333-355), decided on
 * the device in block order without a host round trip and without one SHT per
 * block: the per-block map changes come from one shared-recurrence block
 * synthesis and one weighted Gram pass.  F = 1 (T) or 2 (EB).
 * blk [F][lmax+1]: block (0..K-1, decision order: spectra in MH order) of each
 * (field, l), -1 outside every block; blk_lmax [K]: largest l of each block
 * (-1: empty); blk_field [K]; blk_bins [2K]: bin range [lo, hi) of each block;
 * s_nc [F][(lmax+1)^2]; dl_cur / dl_prop [F][lmax+1]: unbinned current and
 * proposed D_l; logr / prop_binned / binned [F][maxbins] (binned in/out:
 * accepted blocks take the proposal's bins); u_acc [K * n_iter] accept
 * uniforms in decision order; accept_out [K * n_iter]. */
int gs_masked_pixel_mh(gs_masked* ctx, int K, int n_iter, int maxbins, const int* blk, const int* blk_lmax,
                       const int* blk_field, const int* blk_bins, const double* s_nc, const double* dl_cur,
                       const double* dl_prop, const double* logr, const double* u_acc, const double* prop_binned,
                       double* binned, int32_t* accept_out, void* stream);

/* Gaussian sky draw for synthetic data (the synalm + smoothalm half of
 * healpy.synfast, main_polarization.py:38): alm[f] = beam[f][l] * (C_l^1/2 z)[f]
 * per real slot.  cl [nspec][lmax+1] is C_l (not D_l): nfields 1: TT;
 * 2: EE, BB; 3: TT, EE, BB, TE (TEB uses the Cholesky factor of the (T, E)
 * block).  beam [nfields][lmax+1]; z [nfields][(lmax+1)^2] unit normals
 * supplied by the caller; alm [nfields][(lmax+1)^2].  Device pointers. */
int gs_synalm(int lmax, int nfields, const double* cl, const double* beam, const double* z, double* alm,
              void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GIBBS_CAPI_H */
