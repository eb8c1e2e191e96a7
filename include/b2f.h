/*
 * b2f.h -- C ABI of the MI355X (gfx950) BLAKE2f Table16 witness-fill and constraint-eval
 * engine. Plain pointers and sizes only; no torch or HIP types in the signatures
 * (`stream` is an opaque hipStream_t, NULL = the default stream).
 *
 * Drop-in point: the reference's gadget boundary `Blake2fInstructions<F>`
 * (blake2f-circuit/src/blake2f.rs:40-72), implemented by `Table16Chip`
 * (blake2f-circuit/src/blake2f/table16.rs:338-384), whose region drivers
 * `CompressionConfig::{initialize_with_iv, initialize_with_state, compress, digest}`
 * (table16/compression.rs:1078-1149) assign the trace cell by cell; and the batch entry the
 * reference sketches, `Blake2fChip::construct(config, Vec<Blake2fWitness>)` +
 * `chip.load(&mut layouter)` checked by `MockProver::run(k, ..).verify()`
 * (blake2f.rs:250-303, commented out there). One b2f_fill call assigns every region of a
 * batch of independent compressions; one b2f_eval call is the MockProver check of the
 * resulting trace. The trace contract is docs/LAYOUT.md (LAYOUT v1).
 *
 * Threading: one context per device, externally synchronized, and used on ONE stream at a
 * time: a context owns per-call scratch (half-round states, tile index, lookup scratch) that
 * every stream-ordered call reuses, so two `*_dev` calls of one context in flight on two
 * streams race on it. Use one context per concurrent stream. `*_dev` calls are
 * stream-ordered and asynchronous; b2f_sync() waits and returns any device-side error raised
 * since the previous b2f_sync (errors are sticky until then). Host-pointer calls block. No
 * call aborts; errors come back as B2F_* status codes with a message in b2f_last_error().
 * They map onto halo2's plonk::Error at a Rust call site: B2F_ERR_ROWS ->
 * NotEnoughRowsAvailable, the others -> Synthesis.
 */
#ifndef B2F_H
#define B2F_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define B2F_API __attribute__((visibility("default")))

#define B2F_NUM_ADVICE 10      /* a_0..a_9, table16.rs:281-309 */
#define B2F_NUM_GATES 16       /* selector bits, docs/LAYOUT.md §4 */
#define B2F_CODE_LOOKUP 16
#define B2F_CODE_COPY 17
#define B2F_CODE_FIXED 18   /* fixed-column cell differs from the keygen structure */
#define B2F_CODE_LAYOUT 19  /* the row map was rejected: nothing was checked */
#define B2F_CODE_CHECK 20   /* an internal cross-check failed (B2F_ERR_CHECK, a library defect):
                               the verdict is not trustworthy, whatever the witness */
#define B2F_MAX_ROUNDS (1u << 20)

/* Status codes */
#define B2F_OK 0
#define B2F_ERR_ARG 1       /* null pointer, misaligned buffer, total_rows % 4 != 0 */
#define B2F_ERR_ROUNDS 2    /* rounds > B2F_MAX_ROUNDS */
#define B2F_ERR_ROWS 3      /* buffers hold fewer rows than the batch needs */
#define B2F_ERR_HIP 4       /* HIP runtime error */
#define B2F_ERR_LAYOUT 5    /* offsets are not the prefix sums of R(rounds_i) */
#define B2F_ERR_INPUT 6     /* malformed EIP-152 input (length != 213 or f not 0/1) */
#define B2F_ERR_FIELD 7     /* (at b2f_sync) a grand product's denominator product is zero: a
                               challenge collides with a cell value, its z column is meaningless */
#define B2F_ERR_CHECK 8     /* (at b2f_sync) an internal cross-check failed -- a library defect:
                               the lookup's permuted columns do not multiply to the product of
                               its input columns (its columns are wrong), or the fused pass's
                               long-instance segment list overflowed (its verdict reads unclean) */

/* One EIP-152 compression: the reference's Blake2fWitness{rounds, h, m, t, f}
 * (blake2f.rs:208-239), 216 bytes, naturally aligned. f must be 0 or 1. */
typedef struct {
    uint64_t h[8];
    uint64_t m[16];
    uint64_t t[2];
    uint32_t rounds;
    uint32_t f;
} b2f_input;

/* MockProver-equivalent verdict (docs/LAYOUT.md §6). first_failure = min over all failures
 * of (row << 8) | code (code = selector bit 0..15, B2F_CODE_LOOKUP, B2F_CODE_COPY,
 * B2F_CODE_FIXED), UINT64_MAX when every constraint holds.
 * fixed_failures: rows whose fixed cell (selector mask | k_0 << 16) differs from the one the
 * keygen structure of the row map puts there (b2f_fill_fixed_dev): halo2 fixes selectors and
 * constants at keygen, so a trace checked under a caller-altered fixed column is rejected even
 * when its advice is consistent with the altered selectors.
 * A rejected row map (B2F_ERR_LAYOUT) leaves rows_checked = 0 and first_failure =
 * B2F_CODE_LAYOUT: the report never reads clean for a batch that was not checked. A failed
 * internal cross-check (B2F_ERR_CHECK) does the same with B2F_CODE_CHECK, so a library defect
 * never reads as a witness layout failure. */
typedef struct {
    uint64_t gate_failures[B2F_NUM_GATES];
    uint64_t lookup_failures;
    uint64_t copy_failures;
    uint64_t first_failure;
    uint64_t rows_checked;
    uint64_t fixed_failures;
} b2f_eval_report;

typedef struct b2f_ctx b2f_ctx;

B2F_API int b2f_version(void);

/* Rows of one instance, R(rounds) = 228 + 416*rounds (LAYOUT.md §5). Replaces the SHA row
 * map of compression_util.rs:32-205. Returns 0 when rounds > B2F_MAX_ROUNDS. */
B2F_API uint64_t b2f_layout_rows(uint32_t rounds);

/* offsets[0..n]: row offset of every instance region, i.e. where each `assign_region` of
 * compression.rs:1084/1120/1140 lands in the batch. Host function. */
B2F_API int b2f_layout_offsets(const b2f_input* in, size_t n, uint64_t* offsets);

/* halo2 advice-column index of a_i in the reference's allocation order
 * (table16.rs:281-294: a_5, a_3, a_4, a_6, a_7, a_8, a_9, a_0, a_1, a_2); -1 if i > 9. */
B2F_API int b2f_halo2_column_index(int a_i);

/* Parse one 213-byte EIP-152 precompile input (rounds u32 BE | h 64 B | m 128 B | t 16 B |
 * f 1 B; words little-endian), the format of the reference KAT (blake2f.rs:193-247). */
B2F_API int b2f_parse_eip152(const uint8_t* raw, size_t len, b2f_input* out);

/* Context bound to one HIP device (owns scratch, events, the device status words). */
B2F_API b2f_ctx* b2f_create(int device);
B2F_API void b2f_destroy(b2f_ctx* ctx);
B2F_API const char* b2f_last_error(const b2f_ctx* ctx);

/* Witness fill, device pointers. Replaces CompressionConfig::{initialize_with_iv,
 * compress, digest} (compression.rs:1078-1149) with their helpers
 * (compression_util.rs:208-890, subregion_initial.rs:11-155, SpreadVar::with_lookup
 * spread_table.rs:257-285, AssignedBits::assign_bits table16.rs:136-167) for n instances.
 *   d_in        n records (16-B aligned)
 *   d_offsets   n+1 row offsets (b2f_layout_offsets)
 *   total_rows  rows of the buffers (>= offsets[n], multiple of 4); rows past offsets[n]
 *               are written as zeros
 *   d_advice    column-major uint32 [10][total_rows] (16-B aligned); cell a_c of row r at
 *               d_advice[c * total_rows + r]
 *   d_fixed     uint32 [total_rows]: selector mask (bits 0..15) | constant k_0 << 16
 *   d_h_out     n * 8 uint64 compression outputs h' (may be NULL)
 * Asynchronous on `stream`. */
B2F_API int b2f_fill_dev(b2f_ctx* ctx, const b2f_input* d_in, size_t n,
                         const uint64_t* d_offsets, uint64_t total_rows, uint32_t* d_advice,
                         uint32_t* d_fixed, uint64_t* d_h_out, void* stream);

/* Constraint evaluation over a trace, device pointers: the `MockProver::verify` of
 * blake2f.rs:301-302 -- every gate of compression.rs:604-1056 (as re-derived in
 * LAYOUT.md §4), the spread lookup of spread_table.rs:443-453 on every row, and every
 * copy constraint (`copy_advice`). d_report is overwritten. Asynchronous on `stream`. */
B2F_API int b2f_eval_dev(b2f_ctx* ctx, const uint32_t* d_advice, const uint32_t* d_fixed,
                         const uint64_t* d_offsets, size_t n, uint64_t total_rows,
                         b2f_eval_report* d_report, void* stream);

/* Fused witness fill + constraint evaluation, device pointers: the same trace, h' and
 * verdict as b2f_fill_dev followed by b2f_eval_dev on that trace (MockProver::run then
 * ::verify, blake2f.rs:301-302), in one pass: every cell is checked while it is still on the
 * CU, so the trace is written once and never read back. Arguments as b2f_fill_dev plus the
 * report (overwritten). Asynchronous on `stream`. */
B2F_API int b2f_fill_eval_dev(b2f_ctx* ctx, const b2f_input* d_in, size_t n,
                              const uint64_t* d_offsets, uint64_t total_rows, uint32_t* d_advice,
                              uint32_t* d_fixed, uint64_t* d_h_out, b2f_eval_report* d_report,
                              void* stream);

/* Test hook for the fused path: XOR `mask` into cell (row, col) as b2f_fill_eval_dev assigns
 * it (col 0..9 = a_col, 10 = the fixed column), so both the trace it writes and the trace it
 * checks carry the fault; row = UINT64_MAX turns it off (the default). Lets tests prove the
 * fused verdict equals b2f_eval_dev's / the oracle's on the trace actually written. */
B2F_API int b2f_debug_inject(b2f_ctx* ctx, uint64_t row, uint32_t col, uint32_t mask);

/* Test hook: which path the last b2f_eval_dev call of `ctx` took, after a device synchronize:
 * *out = 0 the fast clean-check pass found the trace clean (its report stands), 1 the pass
 * flagged something and the exact eval kernel wrote the report, 2 no fast pass ran (the exact
 * kernel alone). Lets tests prove a clean trace costs the fast pass only. */
B2F_API int b2f_debug_eval_path(b2f_ctx* ctx, uint32_t* out);

/* Diagnostics: eval-kernel phase cycle totals (s_memtime deltas summed over workgroups) of
 * the EVAL_CLOCK variant since the previous call; out[8 * wave + phase], phases:
 * stage+lookups, barrier 1, prefetch issue, G-table build, gate pass, copies, per-quad paths,
 * barrier 2. That variant exists only in the diagnostics build of this ABI (libb2f_diag.so,
 * selected there by B2F_DIAG_EVAL=23); the product library (libb2f.so) reads no environment,
 * launches only the full kernels and returns zeros here. Clears the totals. */
B2F_API int b2f_debug_clock(b2f_ctx* ctx, uint64_t* out);

/* Keygen structure (halo2 keygen_vk / keygen_pk over Value::unknown() witnesses,
 * benchmarking/src/blake2f_circuit_bench.rs:54-55; SURVEY.md §8(b) "Semantics to preserve"):
 * the fixed column of a batch from its row map alone, no witness -- selector masks and the
 * IV constants k_0 (LAYOUT.md §4/§5), zeros past offsets[n]. Equal to the d_fixed that
 * b2f_fill_dev writes for any witness of the same rounds. B2F_ERR_LAYOUT (at b2f_sync) for an
 * invalid row map. d_fixed 16-byte aligned, total_rows a multiple of 4. Asynchronous. */
B2F_API int b2f_fill_fixed_dev(b2f_ctx* ctx, const uint64_t* d_offsets, size_t n,
                               uint64_t total_rows, uint32_t* d_fixed, void* stream);

/* The copy constraints (equality pairs, `copy_advice` sites: table16.rs:431-433,
 * compression_util.rs:398-416,548-574) of one instance of `rounds` rounds, as keygen records
 * them: writes min(count, cap) quadruples (dst_row, dst_col, src_row, src_col), rows relative
 * to the instance, columns a_0..a_9 (b2f_halo2_column_index maps them to halo2's order), and
 * returns count = 24 + 576 * rounds + 96 (0 if rounds > B2F_MAX_ROUNDS). Host function. */
B2F_API uint64_t b2f_copy_constraints(uint32_t rounds, uint32_t* out4, uint64_t cap);

/* Wait for `stream` and return the first device-side error of the calls issued since the
 * previous b2f_sync (B2F_ERR_LAYOUT / B2F_ERR_ROUNDS from fill/eval, B2F_ERR_FIELD from the
 * lookup / permutation grand products), then clear it. */
B2F_API int b2f_sync(b2f_ctx* ctx, void* stream);

/* Host-pointer conveniences (allocate, copy, run, copy back; blocking). b2f_fill sizes the
 * trace to exactly offsets[n] rows; advice must hold 10*offsets[n] and fixed offsets[n]. */
B2F_API int b2f_fill(b2f_ctx* ctx, const b2f_input* in, size_t n, uint32_t* advice,
                     uint32_t* fixed, uint64_t* h_out);
B2F_API int b2f_eval(b2f_ctx* ctx, const uint32_t* advice, const uint32_t* fixed,
                     const uint64_t* offsets, size_t n, uint64_t total_rows,
                     b2f_eval_report* report);

/* Multi-block chaining (the reference gadget's Blake2f::update /
 * finalize, blake2f.rs:101-168): writes the b2f_input records of one block step for messages
 * 0 .. n-1 -- h from the previous step's outputs h' (d_h_prev, n x 8; the initial state for the
 * first block), the block's 16 message words (d_blocks, n x 16), the byte counter after the
 * block (d_t, n x 2), the final-block flag (d_f, n; non-zero = 1) and `rounds` (12 for
 * BLAKE2b). A host orders its messages by block count so that the messages still running at
 * a step are a prefix (b2f/hasher.py). Asynchronous on `stream`. */
B2F_API int b2f_chain_inputs_dev(b2f_ctx* ctx, const uint64_t* d_h_prev, const uint64_t* d_blocks,
                                 const uint64_t* d_t, const uint32_t* d_f, uint32_t rounds,
                                 size_t n, b2f_input* d_out, void* stream);

/* Fp export: advice cells as elements of the prover's scalar field,
 * the form halo2's prover keeps its advice columns in. Two fields:
 *   pallas::Base (pasta_curves 0.5.1 Fp, halo2_proofs 0.3.0's own field),
 *     p = 0x40000000000000000000000000000000224698fc094cf91b992d30ed00000001;
 *   BN254 Fr (halo2curves 0.3.2 bn256::Fr, the field of the reference's circuit test and KZG
 *     bench: blake2f.rs:283,293, blake2f_circuit_bench.rs:10,34),
 *     r = 0x30644e72e131a029b85045b68181585d2833e84879b9709143e1f593f0000001.
 * Rows [row_begin, row_begin + nrows) of the ten advice columns are written in halo2 column
 * order (b2f_halo2_column_index): element of a_i at row row_begin + r goes to
 * d_out[(h * out_rows + r) * 4 + limb], h = b2f_halo2_column_index(i), 4 little-endian u64
 * limbs. out_rows >= nrows is the column stride (rows past nrows are not written; a prover
 * zero-fills to 2^k). `form`:
 *   B2F_FP_MONTGOMERY        x * 2^256 mod p (the in-memory Fp of pasta_curves)
 *   B2F_FP_CANONICAL         x as a 32-byte little-endian integer (PrimeField::to_repr)
 *   B2F_FP_BN254_MONTGOMERY  x * 2^256 mod r (the in-memory bn256::Fr of halo2curves)
 *   B2F_FP_BN254_CANONICAL   x as a 32-byte little-endian integer
 * (bit 1 selects the field, bit 0 Montgomery form). d_out must be 16-byte aligned.
 * Asynchronous on `stream`. */
#define B2F_FP_CANONICAL 0
#define B2F_FP_MONTGOMERY 1
#define B2F_FP_BN254_CANONICAL 2
#define B2F_FP_BN254_MONTGOMERY 3
B2F_API int b2f_export_fp_dev(b2f_ctx* ctx, const uint32_t* d_advice, uint64_t total_rows,
                              uint64_t row_begin, uint64_t nrows, uint32_t form,
                              uint64_t* d_out, uint64_t out_rows, void* stream);

/* The spread table as the prover's table columns (SpreadTableChip::load, spread_table.rs:470-508;
 * rows from SpreadTableConfig::generate, spread_table.rs:574-600): column c = 0 tag, 1 dense,
 * 2 spread, row x < 2^16 holds (tag(x), x, spread(x)), rows 2^16 .. usable_rows - 1 the
 * layouter's fill_from_row default (row 0's values: zero). Written to
 * d_out[(c * out_rows + row) * 4 + limb] in `form` (any B2F_FP_*), 2^16 <= usable_rows < 2^32,
 * out_rows >= usable_rows, d_out 16-byte aligned. Keygen data (halo2 fixes it in the proving
 * key); the lookup-columns call computes the compressed table internally. Asynchronous. */
B2F_API int b2f_spread_table_dev(b2f_ctx* ctx, uint64_t usable_rows, uint32_t form, uint64_t* d_out,
                                 uint64_t out_rows, void* stream);

/* Lookup-argument prover columns of the spread lookup
 * (spread_table.rs:443-453), as halo2_proofs 0.3.0's lookup prover builds them
 * (plonk/lookup/prover.rs: commit_permuted, permute_expression_pair, commit_product), for
 * n_circuits circuits cut from the trace: circuit c covers trace rows d_row_begin[c] ..
 * + usable_rows - 1 (rows past total_rows read as zero rows, i.e. table row 0), and the
 * table columns hold the 2^16 spread-table rows then the row-0 default up to usable_rows
 * (the layouter's fill_from_row). usable_rows = 2^k - blinding_factors - 1 is the caller's,
 * in [2^16, 2^31]. Challenges theta, beta, gamma: canonical field elements (4 LE u64 limbs).
 * Output, per circuit c and column j, d_out[((c * 5 + j) * out_rows + row) * 4 + limb]:
 *   j = 0  A:  compressed input   theta^2 a_0 + theta a_1 + a_2   (rows < usable_rows)
 *   j = 1  S:  compressed table                                     (rows < usable_rows)
 *   j = 2  A': permuted input (ascending canonical order)           (rows < usable_rows)
 *   j = 3  S': permuted table (A'[i] == S'[i] or A'[i] == A'[i-1])  (rows < usable_rows)
 *   j = 4  z:  lookup grand product, z[0] = 1                       (rows <= usable_rows)
 * in `form` (any B2F_FP_* form: pasta Fp or BN254 Fr, Montgomery or canonical; the
 * challenges are canonical elements of that field); out_rows >= usable_rows + 1, blinding
 * rows are the prover's. d_first_bad[c] receives the first circuit row whose (a_0, a_1, a_2)
 * is not a table row (halo2's ConstraintSystemFailure), UINT64_MAX if none; that circuit's
 * columns are then meaningless. Asynchronous on `stream`. */
B2F_API int b2f_lookup_columns_dev(b2f_ctx* ctx, const uint32_t* d_advice, uint64_t total_rows,
                                   const uint64_t* d_row_begin, uint32_t n_circuits,
                                   uint64_t usable_rows, const uint64_t theta[4],
                                   const uint64_t beta[4], const uint64_t gamma[4], uint32_t form,
                                   uint64_t* d_out, uint64_t out_rows, uint64_t* d_first_bad,
                                   void* stream);

/* Keygen's permutation mapping of one instance of `rounds` rounds (halo2_proofs 0.3.0
 * plonk/permutation/keygen.rs Assembly::copy replayed over b2f_copy_constraints in synthesis
 * order, each copy as copy(destination, source)): for permutation column j (= a_{j+1}, the
 * enable_equality order of table16.rs:312-314) and instance row i < R = b2f_layout_rows(rounds),
 * out[j * R + i] = (c' << 29) | r' names the cell the permutation maps (j, i) to. Writes
 * min(8 R, cap) words, returns 8 R (0 for rounds > B2F_MAX_ROUNDS). Host function. */
B2F_API uint64_t b2f_permutation_mapping(uint32_t rounds, uint32_t* out, uint64_t cap);

/* Permutation-argument prover columns (halo2_proofs 0.3.0 plonk/permutation: build_pk's
 * permutation polynomials and prover.rs commit) of the equality columns a_1..a_8 for one
 * circuit made of the instances with host row map h_offsets[0..n] (trace rows of the batch in
 * d_advice; circuit row = trace row - h_offsets[0]), in a domain of 2^k rows:
 *   d_sigma (nullable): sigma_j(w^i) = delta^c' w^r' for (c', r') the mapped cell, at
 *     d_sigma[(j * out_rows + i) * 4 + limb], j < 8, every row i < 2^k (identity past the
 *     instances);
 *   d_z: for each set c of chunk_len columns (cs.degree() - 2 in halo2) the grand product
 *     z_c[0] = z_{c-1}[usable_rows] (1 for c = 0),
 *     z_c[i + 1] = z_c[i] prod_{j in c} (v_j(i) + beta delta^j w^i + gamma)
 *                          / (v_j(i) + beta sigma_j(w^i) + gamma),   i < usable_rows,
 *     at d_z[(c * out_rows + i) * 4 + limb], rows 0 ..= usable_rows (the blinding rows after
 *     them are the prover's). v_j(i) is the cell of a_{j+1} (zero past the instances).
 * usable_rows = 2^k - blinding_factors - 1 >= h_offsets[n] - h_offsets[0]; omega = the
 * domain's generator (F::ROOT_OF_UNITY squared S - k times), delta = F::DELTA, beta, gamma:
 * canonical elements of the field chosen by `form` (any B2F_FP_*; outputs in that form).
 * out_rows >= usable_rows + 1 (and >= 2^k with d_sigma); 16-byte aligned outputs. A valid
 * trace closes: z_last[usable_rows] = 1. Asynchronous on `stream` after a short host setup
 * (mapping patterns cached per rounds in the context; the instance table goes up by an async
 * copy from pinned staging). The host waits only for the previous call's table upload, and for
 * the whole stream only when a device buffer has to grow (a new `rounds`, more instances, a
 * larger k or a smaller chunk_len than before). Scratch: ceil(8 / chunk_len) column sets of
 * 3 x 32 B per usable row plus O(2^k / 1024) tables. */
B2F_API int b2f_permutation_columns_dev(b2f_ctx* ctx, const uint32_t* d_advice, uint64_t total_rows,
                                        const uint64_t* h_offsets, size_t n, uint32_t k,
                                        uint64_t usable_rows, const uint64_t omega[4],
                                        const uint64_t delta[4], const uint64_t beta[4],
                                        const uint64_t gamma[4], uint32_t chunk_len, uint32_t form,
                                        uint64_t* d_sigma, uint64_t* d_z, uint64_t out_rows,
                                        void* stream);

/* Keygen's permutation polynomials alone (halo2_proofs 0.3.0 plonk/permutation/keygen.rs
 * build_pk: the sigma columns depend on the circuit's structure, not on a witness): the same
 * d_sigma that b2f_permutation_columns_dev writes for the row map h_offsets[0..n], domain 2^k,
 * omega, delta and `form` -- sigma_j(w^i) = delta^c' w^r' at d_sigma[(j * out_rows + i) * 4 +
 * limb], j < 8, every row i < 2^k. A prover computes it once per circuit shape and then calls
 * b2f_permutation_columns_dev with d_sigma = NULL per proof (the z columns never read sigma).
 * h_offsets[n] - h_offsets[0] < 2^k, out_rows >= 2^k, d_sigma 16-byte aligned. Asynchronous on
 * `stream` after the same short host setup. */
B2F_API int b2f_permutation_sigma_dev(b2f_ctx* ctx, const uint64_t* h_offsets, size_t n, uint32_t k,
                                      const uint64_t omega[4], const uint64_t delta[4], uint32_t form,
                                      uint64_t* d_sigma, uint64_t out_rows, void* stream);

/* Per-kernel timing with HIP events recorded on the launch stream around every kernel the
 * fill/eval calls launch (no host synchronization while recording). b2f_set_timing(ctx, 1)
 * clears the log and starts recording; b2f_kernel_times waits for the recorded events and
 * returns, per kernel kind, the summed duration (ms) and the launch count, then clears the
 * log. Kinds: */
#define B2F_KERNEL_RECORD 0 /* BLAKE2f compression + half-round states (fill, part 1) */
#define B2F_KERNEL_FILL 1   /* trace expansion (fill, part 2) */
#define B2F_KERNEL_EVAL 2   /* constraint evaluation */
#define B2F_KERNEL_EXPORT 3 /* Fp export */
#define B2F_KERNEL_FILL_EVAL 4 /* fused trace expansion + constraint evaluation */
#define B2F_KERNEL_LOOKUP 5 /* lookup-argument prover columns (all passes of one call) */
#define B2F_KERNEL_PERM 6   /* permutation-argument prover columns (all passes of one call) */
#define B2F_KERNEL_PERM_SIGMA 7 /* permutation keygen: the sigma columns (b2f_permutation_sigma_dev) */
#define B2F_NUM_KERNELS 8
/* total_ms and count must each hold b2f_num_kernels() entries (= B2F_NUM_KERNELS of the
 * header the library was built with; it grew from 7 to 8 with B2F_KERNEL_PERM_SIGMA): a caller
 * built against another header sizes its buffers from the query, so the library never writes
 * past them. */
B2F_API int b2f_num_kernels(void);
B2F_API int b2f_set_timing(b2f_ctx* ctx, int enable);
B2F_API int b2f_kernel_times(b2f_ctx* ctx, double* total_ms, uint32_t* count);

#ifdef __cplusplus
}
#endif
#endif /* B2F_H */
