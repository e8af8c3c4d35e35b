/* clyload.h — NewCouloyDB's index load on the device, from data files on disk
 * (libclyscan.so; couloydb_amd/csrc/clyload.hip).
 *
 * Replaces NewCouloyDB -> loadDataFile -> loadIndexFromHintFile -> loadIndex
 * (db.go:44-115, 442-485, 487-655; merge.go:240-287) up to "index built":
 *   - the directory's data files: every entry named `*.cly` whose stem (the
 *     name up to its first '.') strconv.Atoi parses (any other such name fails
 *     the open with CLY_ERR_DIR, db.go:451-457), fids ascending, the file read
 *     being "%09d.cly" of uint32(fid) (an absent one reads as empty: the
 *     reference creates it empty), the last fid the active file;
 *   - `hint-index` (when present, even without data files): every record's
 *     key -> DecodeLogRecordPos(value) into the String index first
 *     (merge.go:257-287, strIndex.Put of the stored key, whatever its record's
 *     types), so that the data files' String Put/Del records override it;
 *   - `merge-finished` (when present and data files exist): its record at
 *     offset 0 must read (ReadLogRecord) and its value must be an integer
 *     (strconv.Atoi), else the open fails (merge.go:240-255, db.go:492-502);
 *     the data files are read in full either way (db.go:502 discards
 *     deleteLessThan's result);
 *   - the files are mmap'd, copied to the device, scanned (cly_scan_device),
 *     all five indexes rebuilt on the device (cly_index_device: tx
 *     commit/rollback, last writer wins, the TTL sweep at the context's clock,
 *     cly_ctx_set_clock); the host then holds the String, ListMeta, Hash, List
 *     and Set indexes (key -> LogPos) that updateIndex builds in the MemTables
 *     (meta/memTable.go:15-30, index.go);
 *   - the TTL sweep's db.Del (db.go:639-651, 186-215): every String key whose
 *     winning put has expired leaves the index, and its tombstone record
 *     {0x00 || key, LogRecordDeleted} is appended to the active file by
 *     appendLogRecord's rule (a new file fid+1 when WriteOff + size >
 *     DataFileSize); cly_db_open_opts with CLY_DB_APPLY_SWEEP writes those
 *     records to disk (O_APPEND, as the FileIO writer does), and the stats
 *     report the active file and WriteOff after the sweep either way.  The
 *     reference issues the Del calls in Go map order; the library uses scan
 *     order (the set of records and WriteOff agree whenever no rotation falls
 *     between two of them).
 * Read errors fail the open with their status (ErrInvalidCRC etc.), as
 * NewCouloyDB does, in its order: the hint file's (a record that does not
 * read, or whose position does not decode), then merge-finished's, then the
 * data files' in fid order.  Out of scope (the Go caller's): loadMergeFiles' moving of
 * the merge directory (merge.go:195-238), the file lock, and scheduling the TTL
 * jobs of keys that expire later (cly_db_entries lists them with their
 * expiration).                                                                */
#ifndef CLYLOAD_H
#define CLYLOAD_H
#include "clyscan.h"
#ifdef __cplusplus
extern "C" {
#endif

#define CLY_DB_NOT_FOUND 1    /* public.ErrKeyNotFound                           */
#define CLY_DB_EOF       2    /* cly_db_value: ReadLogRecord at pos returned io.EOF */
#define CLY_ERR_DIR     -14   /* "the data dir maybe contaminated or damaged":
                                 a *.cly name whose stem strconv.Atoi rejects   */
#define CLY_ERR_MERGE_FIN -15 /* merge-finished's record at 0 does not read, or
                                 its value is not an integer (getNonMergeFileId) */
#define CLY_ERR_KEY_EMPTY -16 /* public.ErrKeyIsEmpty: the TTL sweep's db.Del of an
                                 expired String key whose realKey is empty
                                 (db.go:186-188, returned by loadIndex db.go:646-649) */

typedef struct cly_db cly_db;
typedef struct cly_load_stats {
    double   list_map_ms;     /* readdir + open + mmap of the data files         */
    double   h2d_ms;          /* files to the device                             */
    double   scan_ms;         /* cly_scan_device                                 */
    double   index_ms;        /* cly_index_device + tables, host records, states back */
    double   insert_ms;       /* host index inserts (the MemTable Put/Del)       */
    double   total_ms;
    uint64_t n_files, bytes, records;
    uint64_t str_keys, listmeta_keys, hash_fields, list_items, set_members;
    uint32_t active_fid;      /* activityFile.FileId after the open (TTL sweep included) */
    uint32_t _pad;
    int64_t  write_off;       /* activityFile.WriteOff after the open (db.go:632-634 + the sweep's appends) */
    uint64_t hint_records;    /* hint-index records loaded                        */
    uint64_t n_expired;       /* String keys the TTL sweep db.Del'd               */
    int64_t  write_off_loaded;/* WriteOff as loadIndex leaves it (before the sweep) */
    uint32_t active_fid_loaded;
    uint32_t sweep_files;     /* new data files the sweep's appends opened        */
    uint32_t n_shards;        /* contexts that loaded files (cly_db_open_multi)   */
    uint32_t _pad2;
    uint64_t tuple_slots;     /* device tuple slots the scans allocated (exact: records + 16 per shard) */
    double   order_ms;        /* the String / ListMeta winners sorted by key on the device (part of index_ms) */
    uint32_t order_rounds;    /* refinement rounds of that sort (keys of 16+ bytes sharing 15-byte prefixes) */
    uint32_t _pad3;
} cly_load_stats;

/* NewCouloyDB's Options the open uses.                                        */
typedef struct cly_db_options {
    uint64_t data_file_size;  /* Options.DataFileSize (0: 256 MiB, options.go:32) */
    uint32_t flags;           /* CLY_DB_APPLY_SWEEP: write the sweep's tombstones */
    uint32_t _pad;
} cly_db_options;
#define CLY_DB_APPLY_SWEEP 1u

/* Optional start-up call of a process that will open databases: allocates
 * the load driver's page-locked staging (16 copy threads x 2 x 8 MiB) now, so
 * that the first open does not (without it each copy thread allocates its
 * pair at first use: 15-25 ms more on a first open).  The current device's
 * context must exist.  Tried once per process; CLY_OK, or CLY_ERR_DEVICE
 * (remembered; the opens still work, allocating lazily).                     */
int  cly_load_prepare(void);
/* cly_db_open = cly_db_open_opts with default options (nothing written).    */
int  cly_db_open(cly_ctx* ctx, const char* dir, cly_db** out, cly_load_stats* st);
int  cly_db_open_opts(cly_ctx* ctx, const char* dir, const cly_db_options* opt, cly_db** out, cly_load_stats* st);
/* The same open over nctx contexts (one per GPU; several may share one): the
 * files (hint-index first, then the data files by fid) are cut into nctx
 * contiguous ranges balanced by bytes, and each context copies its range to
 * its device and scans it (cly_scan_device), all in parallel.  The tuples are
 * then gathered in fid order on ctxs[0]'s device, whose index rebuild reads
 * every range's bytes in place (peer access between devices): loadIndex's
 * single pass over the fids (db.go:582-637) with its tx buffers, so a
 * transaction whose records and commit fall in different ranges resolves as
 * in one pass.  Result identical to cly_db_open_opts(ctxs[0], ...).
 * CLY_ERR_DEVICE when a range's device cannot be reached from ctxs[0]'s.
 * 1 <= nctx <= 16, each context listed once (CLY_ERR_ARG otherwise: a context
 * runs one scan at a time; several contexts may share a device).  The path
 * with contexts on different devices (peer copies of the tuples, peer reads
 * by the index rebuild) has not been run on a multi-GPU node.                */
int  cly_db_open_multi(cly_ctx* const* ctxs, int nctx, const char* dir, const cly_db_options* opt, cly_db** out,
                       cly_load_stats* st);
void cly_db_close(cly_db* db);
/* Index lookups: CLY_OK with *pos, or CLY_DB_NOT_FOUND.                      */
int  cly_db_get(cly_db* db, const uint8_t* key, uint64_t klen, cly_pos* pos);          /* String   */
int  cly_db_listmeta(cly_db* db, const uint8_t* key, uint64_t klen, cly_pos* pos);     /* ListMeta */
int  cly_db_hget(cly_db* db, const uint8_t* key, uint64_t klen, const uint8_t* field, uint64_t flen,
                 cly_pos* pos);                                                         /* Hash     */
int  cly_db_lget(cly_db* db, const uint8_t* key, uint64_t klen, const uint8_t* seq, uint64_t slen,
                 cly_pos* pos);      /* List: getListDataIndex(key).Get(seqBuf), seqBuf = seq.GobEncode() bytes as given */
int  cly_db_sget(cly_db* db, const uint8_t* key, uint64_t klen, const uint8_t* member, uint64_t mlen,
                 cly_pos* pos);      /* Set: getSetIndex(key).Get(hashMemberKey(key, member)) */
/* The index key updateIndex derives (db.go:511-575) for a record of data type
 * dtype from its decoded key bytes d[0:n] (the stored key of a record without
 * a txId, else the realKey): P || R into out (*plen = |P|): String/ListMeta
 * P = "", R = realKey; Hash P = LE32(len key), R = key || field; List
 * P = len || seq.GobEncode(), R = key; Set P = hashMemberKey, R = key.
 * Returns the length, -1 if Go's decode panics, -2 for a data type without an
 * index, -3 if cap is too small.                                             */
int64_t cly_index_key(uint32_t dtype, const uint8_t* d, uint64_t n, uint8_t* out, uint64_t cap, uint32_t* plen);
/* getLogRecordByPos (db.go:680-704): the value of the record at pos into buf
 * (*vlen = its length, 0 on any error; CLY_ERR_CAPACITY if cap is too small).
 * CLY_DB_NOT_FOUND when pos.Fid is not a data file of the db or the record is
 * a LogRecordDeleted; CLY_DB_EOF when ReadLogRecord returns io.EOF there;
 * CLY_ERR_CRC on a checksum mismatch; CLY_ERR_OFFSET for a negative offset;
 * the panics' codes (CLY_ERR_TRUNC5, CLY_ERR_VARINT).                        */
int  cly_db_value(cly_db* db, const cly_pos* pos, uint8_t* buf, uint64_t cap, uint64_t* vlen);

/* Enumeration of what the load produced (for bulk-loading the caller's
 * MemTables and TTL queue).  Pointers stay valid until cly_db_close.  The
 * order is the reference BTree's (meta/btree.go:64-66, bytes.Compare): String
 * and ListMeta entries ascending by key (sorted on the device during the
 * open); Hash / List / Set entries grouped by key, the keys ascending, and
 * inside a key ascending by sub (field, seq gob bytes, member hash) — each
 * group is one getHashIndex(key) / getListDataIndex / getSetIndex MemTable.
 * CLY_IT_EXPIRED keeps the sweep's order.  Not thread-safe.                  */
#define CLY_IT_STRING   0     /* key = realKey, pos, expiration (0 = none; else the
                                 UnixNano the reference's ttl job fires at)   */
#define CLY_IT_LISTMETA 1     /* key, pos                                       */
#define CLY_IT_HASH     2     /* key, sub = field, pos                          */
#define CLY_IT_LIST     3     /* key, sub = seq.GobEncode() bytes, pos          */
#define CLY_IT_SET      4     /* key, sub = hashMemberKey (4 B), pos            */
#define CLY_IT_EXPIRED  5     /* key: the String keys the TTL sweep db.Del'd, in
                                 the order their tombstones are appended      */
typedef struct cly_db_entry {
    const uint8_t* key;
    uint64_t       key_len;
    const uint8_t* sub;
    uint64_t       sub_len;
    cly_pos        pos;
    int64_t        expiration;
} cly_db_entry;
uint64_t cly_db_count(cly_db* db, int kind);
/* entries first .. first+n-1 of a kind into out; returns how many were written */
uint64_t cly_db_entries(cly_db* db, int kind, uint64_t first, cly_db_entry* out, uint64_t n);

#ifdef __cplusplus
}
#endif
#endif
