/*
 * asan_driver — runs the CPU restatement (refcpu.c, linked in) over a dump of oracle calls
 * written by tests/test_oracle_asan.py, in a process built with AddressSanitizer,
 * LeakSanitizer and UBSan (oracle/Makefile target `asan`). TEST INFRASTRUCTURE ONLY.
 *
 * Every input array of the dump gets a heap block of exactly its size, so a read past the end
 * of any SoA array the oracle is handed is an ASan report. Each result is printed as one line
 * "<tag> <hash>" (the fold below), which the test compares with the same fold over the results
 * of the normal build (oracle/librefcpu.so through pyoracle), so the sanitized run is also
 * checked for equal answers.
 *
 * Dump: a sequence of ops (u32 code, then operands). A struct operand is
 *   u32 size, size raw bytes (the ctypes struct), u32 n_ptr, n_ptr x { u32 offset, u64 nbytes, bytes }
 * where each record is the array a pointer field at `offset` points to (pointer fields without a
 * record are NULL). An absent optional struct is size 0.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "refcpu.h"

enum { OP_CREATE = 1, OP_CFK, OP_RANGES, OP_REDUNDANT, OP_MISSING, OP_DEPS, OP_RECOVERY, OP_MERGE, OP_PREACCEPT,
       OP_LEVELS, OP_DESTROY };

static FILE* in;
static void* owned[1 << 16];
static int n_owned;

static void die(const char* m)
{
    fprintf(stderr, "asan_driver: %s\n", m);
    exit(2);
}

static void rd(void* p, size_t n)
{
    if (n && fread(p, 1, n, in) != n) die("short read");
}

static uint32_t rd32(void) { uint32_t v; rd(&v, 4); return v; }
static uint64_t rd64(void) { uint64_t v; rd(&v, 8); return v; }

static void* keep(void* p)
{
    if (n_owned == (int)(sizeof(owned) / sizeof(owned[0]))) die("too many blocks");
    return owned[n_owned++] = p;
}

/* a struct operand of `want` bytes, or NULL when the dump holds an absent one */
static void* rd_struct(size_t want)
{
    const uint32_t size = rd32();
    if (size == 0) return NULL;
    if (size != want) die("struct size differs from the header's");
    char* s = keep(malloc(size));
    rd(s, size);
    const uint32_t np = rd32();
    for (uint32_t i = 0; i < np; ++i)
    {
        const uint32_t off = rd32();
        const uint64_t nb = rd64();
        if (off + sizeof(void*) > size) die("pointer offset");
        void* a = keep(malloc(nb ? nb : 1));
        rd(a, nb);
        memcpy(s + off, &a, sizeof(void*));
    }
    return s;
}

/* H = H * FNV_PRIME + sum_i u64(x_i) * (2i + 1) + n, wrapping; signed values sign-extended */
#define FOLD_PRIME 0x100000001b3ull
static uint64_t fold_i64(uint64_t h, const int64_t* a, uint64_t n)
{
    uint64_t s = 0;
    for (uint64_t i = 0; i < n; ++i) s += (uint64_t)a[i] * (2 * i + 1);
    return h * FOLD_PRIME + s + n;
}
static uint64_t fold_u64(uint64_t h, const uint64_t* a, uint64_t n) { return fold_i64(h, (const int64_t*)a, n); }
static uint64_t fold_i32(uint64_t h, const int32_t* a, uint64_t n)
{
    uint64_t s = 0;
    for (uint64_t i = 0; i < n; ++i) s += (uint64_t)(int64_t)a[i] * (2 * i + 1);
    return h * FOLD_PRIME + s + n;
}
static uint64_t fold_u32(uint64_t h, const uint32_t* a, uint64_t n)
{
    uint64_t s = 0;
    for (uint64_t i = 0; i < n; ++i) s += (uint64_t)a[i] * (2 * i + 1);
    return h * FOLD_PRIME + s + n;
}
static uint64_t fold_u8(uint64_t h, const uint8_t* a, uint64_t n)
{
    uint64_t s = 0;
    for (uint64_t i = 0; i < n; ++i) s += (uint64_t)a[i] * (2 * i + 1);
    return h * FOLD_PRIME + s + n;
}

static uint64_t fold_result(const rc_result* r)
{
    uint64_t h = r->n_txns;
    const uint64_t n = r->n_txns;
    for (int m = 0; m < AD_NMAPS; ++m)
    {
        const uint64_t nk = r->keys_off[m][n], nt = r->txn_off[m][n], no = r->k2t_off[m][n];
        h = fold_u64(h, r->keys_off[m], n + 1);
        h = fold_i64(h, r->keys[m], nk);
        if (m == AD_MAP_RANGE) h = fold_i64(h, r->keys_end[m], nk);
        h = fold_u64(h, r->txn_off[m], n + 1);
        h = fold_u64(h, r->txn_msb[m], nt);
        h = fold_u64(h, r->txn_lsb[m], nt);
        h = fold_i32(h, r->txn_node[m], nt);
        h = fold_u64(h, r->k2t_off[m], n + 1);
        h = fold_i32(h, r->k2t[m], no);
    }
    return h;
}

int main(int argc, char** argv)
{
    if (argc != 2) die("usage: asan_driver DUMP");
    in = fopen(argv[1], "rb");
    if (!in) die("open");
    rc_store* st = NULL;
    rc_result* res[256];
    int n_res = 0;
    uint32_t op;
    while (fread(&op, 4, 1, in) == 1)
    {
        int rc = 0;
        switch (op)
        {
            case OP_CREATE:
            {
                const ad_config* cfg = rd_struct(sizeof(ad_config));
                if (st) rc_store_destroy(st);
                rc = rc_store_create(cfg, &st);
                break;
            }
            case OP_CFK: rc = rc_cfk_load(st, rd_struct(sizeof(ad_cfk_soa))); break;
            case OP_RANGES: rc = rc_range_cmds_load(st, rd_struct(sizeof(ad_range_cmds_soa))); break;
            case OP_REDUNDANT: rc = rc_redundant_load(st, rd_struct(sizeof(ad_redundant_soa))); break;
            case OP_MISSING: rc = rc_cfk_missing_load(st, rd_struct(sizeof(ad_cfk_missing_soa))); break;
            case OP_DEPS:
            case OP_RECOVERY:
            {
                const uint32_t arg = rd32();
                const ad_query_soa* q = rd_struct(sizeof(ad_query_soa));
                if (n_res == 256) die("too many results");
                rc = op == OP_DEPS ? rc_deps_batch(st, q, arg, 0, 0, &res[n_res]) : rc_recovery_batch(st, q, arg, 0, 0, &res[n_res]);
                if (!rc) printf("%s %llu\n", op == OP_DEPS ? "deps" : "recovery", (unsigned long long)fold_result(res[n_res++]));
                break;
            }
            case OP_MERGE:
            {
                const uint32_t k = rd32();
                if (k == 0 || (int)k > n_res) die("merge arity");
                rc_result* merged = NULL;
                rc = rc_result_merge((const rc_result* const*)&res[n_res - k], (int)k, &merged);
                if (!rc)
                {
                    printf("merge %llu\n", (unsigned long long)fold_result(merged));
                    rc_result_free(merged);
                }
                break;
            }
            case OP_PREACCEPT:
            {
                const uint32_t permit = rd32();
                const uint64_t epoch = rd64();
                const ad_range_map_soa* mc = rd_struct(sizeof(ad_range_map_soa));
                const ad_range_map_soa* rb = rd_struct(sizeof(ad_range_map_soa));
                const ad_query_soa* q = rd_struct(sizeof(ad_query_soa));
                const uint64_t n = q->n_txns;
                uint64_t* om = keep(calloc(n + 1, 8));
                uint64_t* ol = keep(calloc(n + 1, 8));
                int32_t* on = keep(calloc(n + 1, 4));
                uint8_t* of = keep(calloc(n + 1, 1));
                rc = rc_preaccept(mc, rb, q, permit, epoch, om, ol, on, of);
                if (!rc)
                {
                    uint64_t h = fold_u64(fold_u64(0, om, n), ol, n);
                    h = fold_u8(fold_i32(h, on, n), of, n);
                    printf("preaccept %llu\n", (unsigned long long)h);
                }
                break;
            }
            case OP_LEVELS:
            {
                const ad_graph_soa* g = rd_struct(sizeof(ad_graph_soa));
                uint32_t* lv = keep(calloc(g->n_txns + 1, 4));
                rc = rc_levels(g, lv);
                if (!rc) printf("levels %llu\n", (unsigned long long)fold_u32(0, lv, g->n_txns));
                break;
            }
            case OP_DESTROY:
                for (int i = 0; i < n_res; ++i) rc_result_free(res[i]);
                n_res = 0;
                if (st) rc_store_destroy(st);
                st = NULL;
                break;
            default: die("unknown op");
        }
        if (rc)
        {
            fprintf(stderr, "asan_driver: op %u failed with %d: %s\n", op, rc, st ? rc_last_error(st) : "");
            return 3;
        }
    }
    for (int i = 0; i < n_res; ++i) rc_result_free(res[i]);
    if (st) rc_store_destroy(st);
    for (int i = 0; i < n_owned; ++i) free(owned[i]);
    fclose(in);
    return 0;
}
