// cfk_update.hpp — SURVEY §8 f1: CommandsForKey.update applied to the device-resident snapshot
// (cfk_update.hip). Host launch interface.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "common.hpp"

namespace adx {

// A batch of updates (device pointers; ad_cfk_update_soa).
struct CfkUpdIn {
    uint64_t n;
    const int64_t* keys;
    const uint64_t* txn_msb; const uint64_t* txn_lsb; const int32_t* txn_node;
    const uint64_t* exec_msb; const uint64_t* exec_lsb; const int32_t* exec_node;
    const uint8_t* status;
    // the command's ballot (acceptedOrCommitted) per update; null = Ballot.ZERO for every update
    const uint64_t* bal_msb; const uint64_t* bal_lsb; const int32_t* bal_node;
    // the command's deps on the key per update (partialDeps().txnIds(key) past shardRedundantBefore,
    // ascending): [dep_off[i], dep_off[i+1]); null = none given
    const uint64_t* dep_off; const uint64_t* dep_msb; const uint64_t* dep_lsb; const int32_t* dep_node;
};

// TxnInfo.ballot() of an entry (raw Timestamp fields; zero = Ballot.ZERO)
struct Bal {
    uint64_t msb, lsb;
    int32_t node, pad;
};

// Insertions: an update whose txnId the key's byId does not hold is inserted at its byId position;
// ids the dictionary does not hold join it first (appended when newer than all of them, merged
// with a rank remap otherwise).
// Per-entry state kept on the device beside the derived snapshot (built by the ingest): the
// InternalStatus and executeAt rank of every byId entry and the key index each entry belongs to.
// The derived arrays (ent, cand, cwr, w, krec, kent, trees) are rebuilt from it after an update.
struct CfkDevState {
    uint8_t* status;               // [n_ent]
    uint32_t* xrank;               // [n_ent] executeAt rank
    uint32_t* ekey;                // [n_ent] key index
    uint64_t* dict_lsb_raw;  // [n_dict] raw lsb of every dictionary id (flag-bit identity check)
    Bal* ballot;             // [n_ent] or null: every entry's ballot is Ballot.ZERO
    uint32_t* mref;          // [n_ent] or null: the entry's TxnInfo.missing() list in CfkMiss (MREF_*)
    // derived arrays rewritten in place (the snapshot's const views alias them)
    uint2* ent; KeyRec* krec; KeyEntry* kent;
};

// Output buffers the derivation may grow: returned pointers replace the snapshot's views.
struct CfkDerivedBufs {
    uint32_t* cand; uint64_t cand_cap;
    uint32_t* cwr; uint64_t cwr_cap;
    uint2* w; uint64_t w_cap;
};

// Key-indexed arrays of a snapshot (new keys: spare buffers sized by keys_spare)
struct KeyBufs {
    int64_t* keys; KeyRec* krec; uint32_t* kcell; KeySlot* khash; KeyEntry* kent;
    uint64_t hcap;                 // KeySlot slots (a power of two)
};

// Buffer growth for insertions (owned by the caller; all pointers device memory).
struct CfkGrow {
    void* ctx;
    // dictionary arrays with room for n_new ids, the first n_old kept
    int (*dict)(void* ctx, uint64_t n_old, uint64_t n_new, uint64_t** hi, uint64_t** lo, int32_t** node, uint64_t** lsb_raw);
    // spare per-entry arrays for ne_new entries (ent padded to whole 64-entry frames); *bal only
    // when the store holds ballots (else left null)
    int (*entries)(void* ctx, uint64_t ne_new, uint2** ent, uint8_t** status, uint32_t** xrank, uint32_t** ekey, Bal** bal,
                   uint32_t** mref);
    // make the spare arrays current (commit = true) or current ones spare again (rollback) and size
    // the snapshot's trees for ne entries; returns the now-current arrays
    int (*swap)(void* ctx, uint64_t ne, uint2** ent, uint8_t** status, uint32_t** xrank, uint32_t** ekey, Bal** bal,
                uint32_t** mref);
    // the store's first ballots: a zeroed (Ballot.ZERO) array for ne entries
    int (*ballot_init)(void* ctx, uint64_t ne, Bal** bal);
    // dictionary merge (new ids older than the newest one): spare dictionary arrays for n ids, and
    // making them current (returns the now-current arrays)
    int (*dict_spare)(void* ctx, uint64_t n, uint64_t** hi, uint64_t** lo, int32_t** node, uint64_t** lsb_raw);
    int (*dict_swap)(void* ctx, uint64_t** hi, uint64_t** lo, int32_t** node, uint64_t** lsb_raw);
    // rank-holding arrays outside the per-entry state, rewritten by a merge: range entries' txw,
    // stabbing cells (rid << 32 | txw), redundantBefore watermark ranks
    uint32_t* r_txw; uint64_t n_rtxw;
    uint64_t* cell_ent; uint64_t n_cell_ent;
    uint32_t* rb_wm; uint64_t n_rb;
    uint32_t* m_ids; uint64_t n_mids;      // TxnInfo.missing() ids as ranks (CfkMiss), null: none
    // new keys (a CommandsForKey created by the update): spare key-indexed arrays for nk keys and a
    // key hash of at least 2 nk slots; keys_swap makes them current. kcell: the current per-key
    // stabbing cells (NO_CELL without a stabbing index)
    int (*keys_spare)(void* ctx, uint64_t nk, KeyBufs* b);
    int (*keys_swap)(void* ctx, KeyBufs* b);
    const uint32_t* kcell;
    // optional: the batch's n new keys (device, complete on `st` when called) as soon as they are known, nk
    // keys in all -- the host may start placing them in the KeyLine hash while the batch runs on the device
    void (*keys_added)(void* ctx, const int64_t* keys, uint64_t n, uint64_t nk, hipStream_t st);
};

// TxnInfo.missing() lists on the device (CommandsForKey.java:332-341): list j = ids
// [off[j], off[j+1]) as ranks, ascending; entry e's list is mref[e] (MREF_NONE: NO_TXNIDS;
// MREF_BORN: inserted by the running batch). Maintained by run_cfk_update when `on`: the updates
// with deps statuses then need their deps (CfkUpdIn.dep_*). After a batch every entry's list is its
// own index (mref[e] = e).
constexpr uint32_t MREF_NONE = 0xFFFFFFFFu;
constexpr uint32_t MREF_BORN = 0xFFFFFFFEu;
struct CfkMiss {
    bool on = false;
    uint64_t n_lists = 0;
    uint64_t* off = nullptr;
    uint32_t* ids = nullptr;
    void* ctx = nullptr;
    // spare CSR buffers for n lists / n_ids ids, and making them current (returns the current ones)
    int (*spare)(void* ctx, uint64_t n, uint64_t n_ids, uint64_t** off, uint32_t** ids) = nullptr;
    int (*swap)(void* ctx, uint64_t** off, uint32_t** ids) = nullptr;
};

struct CfkUpdOut {
    uint64_t n_applied = 0;        // entries changed or inserted
    uint64_t n_inserted = 0;       // entries inserted
    uint64_t n_new_ids = 0;        // ids added to the dictionary
    // a dictionary merge: every rank r = 2i+1 became 2(i + #{j : merge_pos[j] <= i}) + 1; the merge
    // stands even when the batch then fails (the store's content is unchanged by it)
    bool merged = false;
    const uint64_t* merge_pos = nullptr;   // device, [n_new_ids] ascending
    bool rederived = false;        // the derived arrays were rebuilt although the batch failed
    // keys the batch created (they stand when the batch then fails: an empty CommandsForKey is no
    // CommandsForKey to every reader): device, sorted, and their lower bounds among the old keys
    uint64_t n_new_keys = 0;
    const int64_t* new_keys = nullptr;
    const uint64_t* key_pos = nullptr;
    bool rolled_back = false;      // the batch failed after it had been applied and was undone
    bool batch_stood = false;      // the explicit batch was applied and stands, whatever came after it
    int64_t failed_update = -1;    // the update a failure names (batch index), -1: none
    uint64_t n_additions = 0;      // TRANSITIVELY_KNOWN entries inserted from deps (Updating.java:235-263)
    // additions below their key's prunedBefore, dropped (removePrunedAdditions) and handed back for
    // Pruning.loadPruned / PostProcess.LoadPruned (Updating.java:111-117,171): device arrays of the
    // work area, valid until the next batch; lp_update = the index of the update whose deps held the id
    uint64_t n_load_pruned = 0;
    const int64_t* lp_keys = nullptr;
    const uint64_t* lp_msb = nullptr;
    const uint64_t* lp_lsb = nullptr;
    const int32_t* lp_node = nullptr;
    const uint64_t* lp_update = nullptr;
    double ms_locate = 0, ms_derive = 0, ms_total = 0;
};

struct CfkUpdWork;
CfkUpdWork* cfk_upd_work_create();
void cfk_upd_work_destroy(CfkUpdWork* w);
// the snapshot was rebuilt outside run_cfk_update: drop state kept between batches
void cfk_upd_work_invalidate(CfkUpdWork* w);

// Applies the batch (AD_E_* on failure with the store unchanged; message in *err).
// `need` is called with the sizes the derived arrays need; it must return buffers at least that
// large (possibly reallocated) in *bufs.
// With miss (non-null, on): the TxnInfo.missing() lists and the deps-derived additions follow
// (Updating.insertOrUpdate, Updating.java:99-470): see run_cfk_update.
int run_cfk_update(CfkUpdWork* w, DevSnapshot& s, CfkDevState& d, const CfkUpdIn& u, CfkDerivedBufs* bufs,
                   int (*need)(void* ctx, uint64_t cand, uint64_t cwr, uint64_t w, CfkDerivedBufs* bufs), void* need_ctx,
                   const CfkGrow& grow, hipStream_t st, CfkUpdOut* out, std::string* err, CfkMiss* miss = nullptr);

// Every derived array (ent.tau, cand, cwr, w, krec's Write fields, kent, trees) of a snapshot whose
// per-entry state was just built (ingest.hip); AD_E_DUP_EXEC with *bad_entry on a duplicate committed
// executeAt (CommandsForKey.java:1439).
int run_cfk_derive_full(CfkUpdWork* w, DevSnapshot& s, CfkDevState& d, CfkDerivedBufs* bufs,
                        int (*need)(void* ctx, uint64_t cand, uint64_t cwr, uint64_t w, CfkDerivedBufs* bufs), void* need_ctx,
                        hipStream_t st, uint64_t* bad_entry, std::string* err);

struct CfkPruneOut {
    uint64_t n_removed = 0;        // entries removed
    uint64_t n_keys_pruned = 0;    // CommandsForKeys whose prunedBefore moved
    double ms_total = 0;
};

// Pruning.maybePrune (Pruning.java:164-199 -> pruneBefore :205-331) for the keys klist[0..nl) (key
// indices, device; null: every key, nl = n_keys); TxnInfo.missing() from miss when it is on (the
// subset test of :239-251), else NO_TXNIDS for every entry.
// Removed entries leave the per-entry arrays (compacted into the spare buffers), the segments and
// prunedBefore follow, and the derived arrays are rebuilt. Ids stay in the dictionary.
int run_cfk_prune(CfkUpdWork* w, DevSnapshot& s, CfkDevState& d, const uint32_t* klist, uint64_t nl, int32_t prune_interval,
                  int64_t min_hlc_delta, CfkDerivedBufs* bufs,
                  int (*need)(void* ctx, uint64_t cand, uint64_t cwr, uint64_t w, CfkDerivedBufs* bufs), void* need_ctx,
                  const CfkGrow& grow, hipStream_t st, CfkPruneOut* out, std::string* err, CfkMiss* miss = nullptr);

struct CfkTruncOut {
    uint64_t n_removed = 0;        // entries removed
    uint64_t n_keys = 0;           // CommandsForKeys that changed (entries left or prunedBefore cleared)
    double ms_total = 0;
};

// CommandsForKey.withRedundantBeforeAtLeast (CommandsForKey.java:1317-1341) of every key to the
// snapshot's RedundantBefore (rb_* views; watermark ranks are dictionary members): the entries below
// the key's shardRedundantBefore leave (compacted into the spare buffers), a prunedBefore at or below
// it is cleared, the derived arrays are rebuilt, and with miss on the kept entries' missing() lists
// lose the ids below it (Utils.removeRedundantMissing). h_pos (host, n_keys; may be null): each key's
// count of removed entries, for host-held lists.
int run_cfk_truncate(CfkUpdWork* w, DevSnapshot& s, CfkDevState& d, CfkDerivedBufs* bufs,
                     int (*need)(void* ctx, uint64_t cand, uint64_t cwr, uint64_t w, CfkDerivedBufs* bufs), void* need_ctx,
                     const CfkGrow& grow, hipStream_t st, CfkTruncOut* out, std::string* err, CfkMiss* miss,
                     uint32_t* h_pos);

// The ids (device arrays, n) join the dictionary where it does not hold them (appended, or merged
// with the rank remap of an update batch: out->merged / merge_pos as run_cfk_update reports them);
// ranks[i] (device) = each id's member rank afterwards. After a merge the derived arrays are derived again
// (out->rederived); the caller rebuilds the KeyLines (cfk_update_follow does).
int run_cfk_dict_ensure(CfkUpdWork* w, DevSnapshot& s, CfkDevState& d, const uint64_t* msb, const uint64_t* lsb,
                        const int32_t* node, uint64_t n, const CfkGrow& grow, CfkDerivedBufs* bufs,
                        int (*need)(void* ctx, uint64_t cand, uint64_t cwr, uint64_t w, CfkDerivedBufs* bufs), void* need_ctx,
                        hipStream_t st, CfkUpdOut* out, uint32_t* ranks, std::string* err);

}  // namespace adx
