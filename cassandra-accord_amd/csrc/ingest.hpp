// ingest.hpp — device-side snapshot ingest (ingest.hip): host launch interface.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <algorithm>
#include <string>

#include "common.hpp"
#include "devmem.hpp"

namespace adx {

// The raw snapshot columns in HBM (ad_cfk_soa as loaded) plus the extra ids the dictionary must
// hold (range command txnIds, RedundantBefore watermarks above NONE).
struct IngestIn {
    uint64_t nk, ne, nx;
    const int64_t* keys;           // [nk] ascending
    const uint64_t* seg;           // [nk + 1]
    const int64_t* pruned;         // [nk] index into the key's byId, -1 none; or null
    const uint64_t* tm; const uint64_t* tl; const int32_t* tn;     // txnIds [ne]
    const uint64_t* em; const uint64_t* el; const int32_t* en;     // executeAts [ne]
    const uint8_t* status;         // [ne]
    const uint64_t* xm; const uint64_t* xl; const int32_t* xn;     // extras [nx]
};

// Outputs (device, caller-sized): the dictionary (normalised words + raw lsb, at most
// ingest_records(in) members), every record's rank, and the per-entry / per-key state of the
// snapshot (CfkDevState: ent.y = txw with ent.x left for the derivation, executeAt rank, key index;
// KeyRec with segment, last txnId and prunedBefore).
struct IngestOut {
    uint64_t* dict_hi; uint64_t* dict_lo; int32_t* dict_node; uint64_t* dict_lsb_raw;
    uint32_t* rec_rank;            // [records]: txnIds [0, ne), differing executeAts, extras last
    uint2* ent; uint32_t* xrank; uint32_t* ekey;
    KeyRec* krec;
    uint64_t n_diff;               // set by ingest_dictionary: the extras' ranks start at ne + n_diff
};

struct IngRec { uint64_t* hi; uint64_t* lo; int32_t* node; uint64_t* lsb; };

using IngDBuf = DevBuf;

struct IngestWork;
IngestWork* ingest_work_create();
void ingest_work_destroy(IngestWork* w);

// upper bound on the dictionary size / records of an ingest
uint64_t ingest_records(const IngestIn& in);
// steps 1-3: dictionary (*n_dict members) and record ranks. AD_E_INCONSISTENT_ID: *bad = a record.
int ingest_dictionary(IngestWork* w, const IngestIn& in, IngestOut& o, hipStream_t st, uint64_t* n_dict, uint64_t* bad,
                      std::string* err);
// step 4: per-entry and per-key state and checks (AD_E_INVAL / AD_E_ORDER, AD_E_STATE: prunedBefore
// outside byId; *bad = the key index).
int ingest_entries(IngestWork* w, const IngestIn& in, const IngestOut& o, hipStream_t st, uint64_t* bad, std::string* err);

// per key: its stabbing cell (cell_E null: NO_CELL) and its KeySlot in the open-addressing key hash
// (hcap slots, a power of two, cleared here)
hipError_t ingest_keys(const int64_t* keys, uint64_t nk, const int64_t* cell_E, uint64_t n_cell_E, int start_inclusive,
                       uint32_t* kcell, KeySlot* khash, uint64_t hcap, hipStream_t st);

}  // namespace adx
