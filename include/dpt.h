/*
 * dpt.h -- C-ABI of the MI355X shortest-tokenization engine (libdpt.so).
 *
 * Drop-in boundary for the reference's DP segmentation path.  The reference has
 * no FFI (pure Python); these entry points are what its Python
 * call surface binds through ctypes (dp-tokenization_amd/dptok/_lib.py):
 *
 *   dpt_vocab_create  <- dp_tokenize_llama's vocabulary capture,
 *                        reference packages/tokenizer_utils.py:53-57
 *                        (t2i = get_vocab(); vocab = set(t2i))
 *   dpt_encode        <- the dp_tokenize closure's per-word loop,
 *                        reference packages/tokenizer_utils.py:66-80, which calls
 *                        compute_shortest_tokenizations (packages/dp_tokenize.py:6-70)
 *                        and obtain_longest_token (packages/dp_tokenize.py:72-84)
 *                        for every word produced by pretokenize_raw
 *                        (packages/tokenizer_utils.py:33-50, DPT_MODE_RAW) or by
 *                        pretokenize_with_llama + merge_tokens
 *                        (packages/tokenizer_utils.py:7-31, DPT_MODE_PRESPLIT)
 *   dpt_token_histogram <- the length comparison of the S2ORC probe,
 *                        reference main_analyze_s2orc.py:269-297 (len(dp_tokenize(x)))
 *   dpt_hist_allreduce <- SURVEY.md §8(b)/(e): the one collective of a sharded corpus (the
 *                        reference is single-process, llama_s2orc.sh:10; no call site there)
 *
 * Conventions: plain pointers and sizes, no C++ exceptions cross this boundary,
 * every function returns an int (0 = DPT_OK, < 0 = error; message in
 * dpt_last_error(), thread-local).  Device-pointer calls are stream-ordered and
 * never synchronise.  A dpt_vocab is immutable after creation and may be shared
 * by threads and streams; a dpt_ctx (workspace) must be used by one stream at a
 * time.
 */
#ifndef DPT_H
#define DPT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DPT_ABI_VERSION 6

/* return codes */
#define DPT_OK 0
#define DPT_E_ARG (-1)      /* bad argument (null pointer, size) */
#define DPT_E_HIP (-2)      /* HIP runtime error */
#define DPT_E_VOCAB (-3)    /* vocabulary not supported (e.g. a token longer than 65535 bytes) */
#define DPT_E_CAP (-4)      /* output capacity too small */
#define DPT_E_NODEV (-5)    /* no HIP device */
#define DPT_E_RCCL (-6)     /* RCCL missing (librccl.so.1 not loadable) or an RCCL call failed (ABI 6) */

/* modes (low 4 bits) */
#define DPT_MODE_RAW 0      /* pretokenize_raw semantics (tokenizer_utils.py:33-50) */
#define DPT_MODE_PRESPLIT 1 /* words start where cut_mask != 0; atoms = code points (llama mode) */
#define DPT_MODE_ATOMS 2    /* caller-defined atoms: cut_mask bit 1 = an atom starts, bit 0 = a word
                               starts (compute_shortest_tokenizations over an arbitrary atom list) */
#define DPT_MODE_MASK 0x0F
/* flags (dpt_dp_host only) */
#define DPT_FLAG_UNCAPPED 0x10 /* inf-initialised DP (inspect_tokenizer.py:77-86): lengths only */
#define DPT_FLAG_LEN_ONLY 0x20 /* capped DP lengths (dp_tokenize.py:70 len_dp[-1]), no ids */

/* per-string status (the reference's exceptions) */
#define DPT_STATUS_OK 0
#define DPT_STATUS_NO_TOKENIZATION 1 /* reference: ipdb.set_trace / ValueError (dp_tokenize.py:84) */
#define DPT_STATUS_EMPTY_WORD 2      /* reference: IndexError (dp_tokenize.py:49) */
#define DPT_STATUS_TOO_LONG 3        /* words, atoms and tokens of any length are exact (the windowed kernels
                                        hand what they cannot hold to the unbounded pass); dpt_encode returns
                                        3 only for a string the unbounded pass's arena could not hold in that
                                        call (dpt_ctx_long_need / dpt_ctx_reserve_vocab); dpt_encode_host and
                                        dpt_dp_host grow the arena and rerun, so they never do */
#define DPT_STATUS_INTERNAL 4        /* engine invariant violated (never expected) */

typedef struct dpt_vocab dpt_vocab;
typedef struct dpt_ctx dpt_ctx;

typedef struct {
    uint32_t n_tokens;     /* entries accepted (non-empty, duplicates collapsed) */
    uint32_t n_nodes;      /* byte-trie nodes */
    uint32_t n_slots;      /* double-array slots (incl. 256 padding) */
    uint32_t max_bytes;    /* longest token, UTF-8 bytes */
    uint32_t max_cp;       /* longest token, code points */
    uint64_t device_bytes; /* device memory held by the vocab */
    uint32_t hash_max_probe;   /* C2's token hash table (ABI 2): buckets a lookup may visit (2: a key's
                                  two choices, round 5); 0 = no table (every selected token is then
                                  re-walked in the trie) */
    uint32_t hash_buckets;     /* its buckets of two entries (0 = no table) */
} dpt_vocab_stats;

const char *dpt_last_error(void);
int dpt_abi_version(void);

/*
 * Build a vocabulary from n_tok UTF-8 strings: token t is
 * utf8_blob[tok_off[t] .. tok_off[t+1]), its id is ids[t] (or t if ids == NULL).
 * Later duplicates win (dict semantics); empty strings are ignored.  The library
 * copies everything, builds a byte double-array trie on the host and uploads it
 * to `device`.
 */
int dpt_vocab_create(const uint8_t *utf8_blob, const uint64_t *tok_off, const int32_t *ids,
                     uint32_t n_tok, int device, dpt_vocab **out);
int dpt_vocab_destroy(dpt_vocab *v);
int dpt_vocab_stats_get(const dpt_vocab *v, dpt_vocab_stats *out);

/* Workspace on `device` (grows on demand; dpt_ctx_reserve makes a later call capture-safe).
 * Device-path workspace per call of n_bytes / n_str: the staged ids (2 bytes per input byte when
 * every vocabulary id is in 0..32767, else 4), 16 bytes per string, and the unbounded pass's arena
 * (20 bytes per input byte it holds; by default max(4 MiB, n_bytes/32) input bytes, at most n_bytes). */
int dpt_ctx_create(int device, dpt_ctx **out);
int dpt_ctx_destroy(dpt_ctx *c);
int dpt_ctx_reserve(dpt_ctx *c, uint64_t n_bytes, uint64_t n_str);   /* both staging widths */
/* Reserve for vocabulary v's staging width (v may be NULL: both) and an unbounded-pass arena holding
 * long_bytes input bytes of long-word strings per call (0: the default above; n_bytes: every string). */
int dpt_ctx_reserve_vocab(dpt_ctx *c, const dpt_vocab *v, uint64_t n_bytes, uint64_t n_str, uint64_t long_bytes);
/* Device bytes held: the device-path workspace and the host path's staging buffers. */
int dpt_ctx_workspace_bytes(const dpt_ctx *c, uint64_t *device_path, uint64_t *host_path);
/* After the ctx's last dpt_encode has completed (synchronise its stream first): the input bytes of the
 * strings its unbounded pass took (*need) and the arena's capacity (*cap).  need > cap: the strings that
 * did not fit have status DPT_STATUS_TOO_LONG -- reserve long_bytes >= need and call again. */
int dpt_ctx_long_need(dpt_ctx *c, uint64_t *need, uint64_t *cap);

/*
 * Tokenize n_str strings, CSR-packed: string s is text[str_off[s]-str_off[0] .. str_off[s+1]-str_off[0]),
 * n_bytes = str_off[n_str] - str_off[0] (passed explicitly so the host never reads device memory).
 * ALL pointers are DEVICE pointers on the ctx's device.  Outputs:
 *   ids[id_off[s] .. id_off[s+1])  token ids of string s (none when status[s] != 0)
 *   id_off[0..n_str]               id_off[0] = 0
 *   status[s]                      DPT_STATUS_*
 *   capped_len[s] (nullable)       sum over words of the reference's len_dp[-1] (dp_tokenize.py:70), -1 if unknown
 * ids_cap must be >= n_bytes (a string never yields more ids than bytes).
 * cut_mask (n_bytes bytes, PRESPLIT and ATOMS only): PRESPLIT: != 0 where a word starts (byte 0 of
 * every string always starts one); ATOMS: bit 1 where an atom starts, bit 0 where a word starts.
 * str_off must be monotone (str_off[s] <= str_off[s+1]) and every string < 4 GiB: the device path
 * cannot check device-resident offsets (an offset that goes backwards reads past the text);
 * dpt_encode_host / dpt_dp_host check both and fail with DPT_E_ARG.
 * Limits: every string < 4 GiB, n_str < 2^31; RAW / PRESPLIT text is UTF-8 (code points are the
 * atoms).  No limit on word, atom or token length: words over 256 bytes take a 2048-byte window
 * pass, longer words (and atoms over 8 bytes, or words over 64 atoms when the vocabulary has
 * tokens over 64 code points) an unbounded one-wave-per-string pass (dpt_long.hip).
 * Stream-ordered on hip_stream (hipStream_t, NULL = default stream); no host synchronisation.
 */
int dpt_encode(dpt_ctx *c, const dpt_vocab *v, int mode, const uint8_t *text, uint64_t n_bytes,
               const uint64_t *str_off, const uint8_t *cut_mask, uint64_t n_str, int32_t *ids,
               uint64_t ids_cap, uint64_t *id_off, int32_t *status, int32_t *capped_len,
               void *hip_stream);

/*
 * dpt_encode without the CSR packing: the ids of string s stay at the string's own byte offset,
 * ids[str_off[s]-str_off[0] + k] for k < counts[s] (uint64 per string; 0 when status[s] != 0) --
 * the layout the tokenize passes write, so the finish pass (offsets + compaction, about 11 % of a
 * cfg2 call) does not run.  For callers that consume per-string id lists -- the dp_tokenize
 * closure's List[int] per string (reference packages/tokenizer_utils.py:66-80) -- rather than
 * one packed array.  Same arguments, limits and stream semantics as dpt_encode; ids_cap >= n_bytes.
 */
int dpt_encode_padded(dpt_ctx *c, const dpt_vocab *v, int mode, const uint8_t *text, uint64_t n_bytes,
                      const uint64_t *str_off, const uint8_t *cut_mask, uint64_t n_str, int32_t *ids,
                      uint64_t ids_cap, uint64_t *counts, int32_t *status, int32_t *capped_len,
                      void *hip_stream);

/* Same with HOST pointers: copies in, runs, copies out, synchronises. */
int dpt_encode_host(dpt_ctx *c, const dpt_vocab *v, int mode, const uint8_t *text, uint64_t n_bytes,
                    const uint64_t *str_off, const uint8_t *cut_mask, uint64_t n_str, int32_t *ids,
                    uint64_t ids_cap, uint64_t *id_off, int32_t *status, int32_t *capped_len);

/*
 * DP by-products without ids (HOST pointers; synchronises).  mode_flags = DPT_MODE_* |
 * DPT_FLAG_LEN_ONLY (capped len_dp[-1] per string, summed over words) or DPT_FLAG_UNCAPPED
 * (minimum token count, 65535 per word that has no tokenization).  status[s] as dpt_encode.
 * edges (nullable, n_bytes entries): for string s and atom end i (1-based atom index within
 * the string) edges[str_off[s]-str_off[0] + i - 1] has bit d set iff atom i-1-d .. i-1 is a
 * token, cost[i-1-d] + 1 == cost[i] and i-1-d is reachable -- the reference's
 * segment_index_dp[i-1] restricted to reachable starts (dp_tokenize.py:40-46), from which the
 * host enumerates every shortest tokenization in the reference's DFS order.
 */
int dpt_dp_host(dpt_ctx *c, const dpt_vocab *v, int mode_flags, const uint8_t *text, uint64_t n_bytes,
                const uint64_t *str_off, const uint8_t *cut_mask, uint64_t n_str, int32_t *status,
                int32_t *lengths, uint64_t *edges);
/*
 * dpt_dp_host with edges, without the 64-atom limit of the masks: an optimal reachable predecessor
 * more than 64 atoms back (a token of more than 64 atoms -- vocabularies with tokens of more than 64
 * code points) is listed in far[] as the pair far[2k] = the edges[] index of the end (str_off[s] -
 * str_off[0] + i - 1), far[2k+1] = the back distance d >= 64 (start i-1-d), in no particular order,
 * instead of status 3.  far_cap counts pairs; *n_far = the pairs found.  Returns DPT_E_CAP (and the
 * needed *n_far) when they do not fit: call again with far_cap >= *n_far.  Replaces the status 3 of
 * reference dp_tokenize.py:40-46's unbounded segment_index_dp (no span limit there).
 */
int dpt_dp_host_far(dpt_ctx *c, const dpt_vocab *v, int mode_flags, const uint8_t *text, uint64_t n_bytes,
                    const uint64_t *str_off, const uint8_t *cut_mask, uint64_t n_str, int32_t *status,
                    int32_t *lengths, uint64_t *edges, uint64_t *far, uint64_t far_cap, uint64_t *n_far);

/*
 * Token-count histogram (device pointers): hist[0..n_bins) counts strings by
 * #ids (last bin = overflow), then hist[n_bins+0] = total ids, hist[n_bins+1] =
 * total strings, hist[n_bins+2+k] = strings with status k (k = 0..4).
 * hist must hold n_bins + 8 int64 and is ACCUMULATED into (zero it first).  2 <= n_bins <= DPT_HIST_MAX_BINS
 * (the bins are counted in LDS).
 */
#define DPT_HIST_MAX_BINS 16384
int dpt_token_histogram(const uint64_t *id_off, const int32_t *status, uint64_t n_str,
                        int64_t *hist, uint32_t n_bins, void *hip_stream);

/*
 * Fold the token-count histogram of dpt_token_histogram into the NEXT dpt_encode call on this ctx
 * (dpt_encode only: dpt_encode_host, dpt_encode_padded and dpt_dp_host* leave it armed; a dpt_encode
 * that fails still consumes it)
 * (its finish pass: no separate launch, no re-read of the offsets and statuses): hist (device
 * pointer, n_bins + 8 int64, layout and accumulate semantics of dpt_token_histogram) is added to
 * once, stream-ordered with that call.  hist NULL cancels.  n_bins above 1024 uses the separate
 * histogram pass after the encode.  One call only: set it again for the next.
 */
int dpt_ctx_set_histogram(dpt_ctx *c, int64_t *hist, uint32_t n_bins);

/* As dpt_ctx_set_histogram; flags DPT_HIST_OVERWRITE: the call's histogram REPLACES hist's contents
 * (the device zeroes it in stream order first) -- a per-step histogram without a memset launch. */
#define DPT_HIST_OVERWRITE 1
int dpt_ctx_set_histogram_ex(dpt_ctx *c, int64_t *hist, uint32_t n_bins, int flags);

/* Per-ctx kernel timing with HIP events on the encode stream (for bench.py's roofline): one event
 * pair per call around the tokenize passes (first pass, 2048-byte pass, unbounded pass). */
int dpt_ctx_profile(dpt_ctx *c, int enable);
/* Sums over calls since the last read (synchronises on the recorded events):
 * ms[0] tokenize passes; ms[1], ms[2] = -1 (not timed); *launches = calls timed. */
int dpt_ctx_profile_read(dpt_ctx *c, double *ms, uint64_t *launches);

/* TEST-ONLY.  Every later call on c starts the unbounded pass's arena counter and the far-pair counter
 * at `bias` instead of 0, with the arena and far-list pointers the kernels get shifted back by as many
 * elements: results are unchanged, but the kernels' arena offsets and far-pair indices are >= bias.
 * With a bias whose low word is >= 2^31 this exercises the 64-bit uniform reassembly of those values
 * (two readfirstlane halves; an int low half sign-extends) without a 40-GiB arena
 * (tests/test_gpu_parity.py::test_long_pass_offsets_past_2g).  bias < 2^62; 0 turns it off. */
int dpt_ctx_debug_counter_bias(dpt_ctx *c, uint64_t bias);

/*
 * Multi-GPU without torch (ABI 6; SURVEY.md §8(b) dpt_hist_allreduce, §8(e) "direct RCCL with a
 * file-store unique id").  One process per GPU: rank 0 calls dpt_rccl_get_unique_id and hands the
 * DPT_RCCL_ID_BYTES bytes to the other ranks by any means (a file, a socket, MPI); every rank then calls
 * dpt_rccl_comm_create with the same id (collective: it blocks until all `world` ranks have joined).
 * RCCL is loaded on first use (dlopen of librccl.so.1: the copy the process already holds -- e.g.
 * PyTorch-ROCm's -- else the one on the library path), so libdpt.so itself does not depend on it;
 * without it these calls return DPT_E_RCCL.
 */
#define DPT_RCCL_ID_BYTES 128
int dpt_rccl_get_unique_id(uint8_t *id_out);
int dpt_rccl_comm_create(const uint8_t *id, int world, int rank, int device, void **comm_out);
int dpt_rccl_comm_destroy(void *rccl_comm);
/*
 * Sum hist[0..n) (device pointer, int64; the dpt_token_histogram layout) over every rank of
 * rccl_comm, in place, stream-ordered on hip_stream (NULL = the default stream): one ncclAllReduce.
 * rccl_comm is an ncclComm_t -- from dpt_rccl_comm_create or the caller's own RCCL setup.
 */
int dpt_hist_allreduce(int64_t *hist, size_t n, void *rccl_comm, void *hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* DPT_H */
