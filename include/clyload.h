/* clyload.h — NewCouloyDB's index load on the device, from data files on disk
 * (libclyscan.so; couloydb_amd/csrc/clyload.hip).
 *
 * Replaces NewCouloyDB -> loadDataFile -> loadIndex (db.go:44-115, 442-485,
 * 487-655) up to "index built": the directory's `%09d.cly` files (fids
 * ascending, the last the active file) are mmap'd, copied to the device,
 * scanned (cly_scan_device) and their String/ListMeta index state rebuilt
 * (cly_index_device, incl. tx commit/rollback and the TTL sweep at the
 * context's clock, cly_ctx_set_clock); the host then holds the String,
 * ListMeta, Hash, List and Set indexes (key -> LogPos) that updateIndex builds
 * in the MemTables (meta/memTable.go:15-30, index.go).
 * A read error of the scan (ErrInvalidCRC etc.) fails the open with its
 * status, as NewCouloyDB does.                                                */
#ifndef CLYLOAD_H
#define CLYLOAD_H
#include "clyscan.h"
#ifdef __cplusplus
extern "C" {
#endif

#define CLY_DB_NOT_FOUND 1    /* public.ErrKeyNotFound                           */

typedef struct cly_db cly_db;
typedef struct cly_load_stats {
    double   list_map_ms;     /* readdir + open + mmap of the data files         */
    double   h2d_ms;          /* files to the device                             */
    double   scan_ms;         /* cly_scan_device                                 */
    double   index_ms;        /* cly_index_device + tuples/states back           */
    double   insert_ms;       /* host index inserts (the MemTable Put/Del)       */
    double   total_ms;
    uint64_t n_files, bytes, records;
    uint64_t str_keys, listmeta_keys, hash_fields, list_items, set_members;
    uint32_t active_fid;      /* activityFile.FileId                             */
    uint32_t _pad;
    int64_t  write_off;       /* activityFile.WriteOff (db.go:632-634)           */
} cly_load_stats;

int  cly_db_open(cly_ctx* ctx, const char* dir, cly_db** out, cly_load_stats* st);
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
 * (*vlen = its length; CLY_ERR_CAPACITY if cap is too small).                */
int  cly_db_value(cly_db* db, const cly_pos* pos, uint8_t* buf, uint64_t cap, uint64_t* vlen);

#ifdef __cplusplus
}
#endif
#endif
