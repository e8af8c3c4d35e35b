/*
 * cly_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of CouloyDB's log-record scan, used as the parity checker
 * (tests/, __graft_entry__.smoke()) and as bench.py's `cpu_baseline` leg.  The
 * product path (libclyscan.so) never links, loads or calls this code.
 *
 * Parity pinning: the reference is Go and no Go toolchain exists in the build
 * container or on the GPU box, so the reference itself cannot be run.  This
 * restatement is pinned by (1) known-answer vectors for the two stdlib pieces it
 * restates (hash/crc32 IEEE check value 0xCBF43926, Go binary.Varint edge cases),
 * (2) the worked record of SURVEY.md §0, and (3) golden fixtures produced by an
 * independent Python restatement built on zlib.crc32 (tests/golden/make_golden.py).
 * The reference ships no byte-level vectors for this path,
 * so byte-level parity with the Go binary itself is "unpinned by the reference".
 */
#ifndef CLY_ORACLE_H
#define CLY_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* identical layout to cly_tuple in include/clyscan.h (48 bytes) */
typedef struct clyo_tuple {
    int64_t  offset, expiration, tx_id;
    uint32_t fid, size, key_size, value_size;
    uint8_t  type, data_type, header_size, txid_len;
    uint32_t crc;
} clyo_tuple;

/* status codes: same values as CLY_END_* / CLY_ERR_* */
enum {
    CLYO_REC = 100,      /* clyo_read_log_record: a record was returned */
    CLYO_END_EOF = 0, CLYO_END_ZERO = 1, CLYO_END_TORN = 2,
    CLYO_ERR_CRC = -1, CLYO_ERR_TRUNC5 = -2, CLYO_ERR_VARINT = -3, CLYO_ERR_OFFSET = -4,
};

/* Go encoding/binary (toolchain >= 1.18, go.mod:3) */
uint64_t clyo_uvarint(const uint8_t* buf, int64_t len, int* n);
int64_t  clyo_varint(const uint8_t* buf, int64_t len, int* n);
int      clyo_put_varint(uint8_t* buf, int64_t x);

/* Go hash/crc32: crc32.Update(crc, IEEETable, p) (ChecksumIEEE = update(0, p)) */
uint32_t clyo_crc32_update(uint32_t crc, const uint8_t* p, size_t len);

/* One ReadLogRecord(offset) call on file bytes F[0..n).  Returns CLYO_REC and
 * fills *t (fid left 0) on success, else a terminal status. */
int clyo_read_log_record(const uint8_t* F, uint64_t n, uint64_t off, clyo_tuple* t);

/* The db.loadIndex inner loop over one file (db.go:590-631): tuples in order.
 * Returns the number of tuples (may exceed cap; only cap are written). */
uint64_t clyo_scan_file(const uint8_t* F, uint64_t n, uint32_t fid,
                        clyo_tuple* out, uint64_t cap,
                        int64_t* end_offset, int32_t* status);

/* EncodeLogRecord (data/logRecord.go:57-84).  Writes into out (capacity >= 26 +
 * klen + vlen) and returns the record size. */
uint64_t clyo_encode_record(uint8_t* out, uint8_t type, uint8_t dtype,
                            const uint8_t* key, uint64_t klen,
                            const uint8_t* val, uint64_t vlen, int64_t expiration);

/* DecodeLogRecordPos (data/logRecord.go:126-134): 0, or CLYO_ERR_VARINT where
 * the reference panics. */
int clyo_decode_pos(const uint8_t* buf, uint64_t len, uint32_t* fid, int64_t* offset);

/* db.merge rewrite loop (merge.go:90-143): live tuples re-encoded with a
 * NO_TX_ID key into merge data files (appendLogRecord rotation, db.go:376-385)
 * plus the hint-index records.  tuple_file[i] indexes bases.  Returns 0,
 * CLYO_ERR_VARINT, -10 (capacity; *res holds the need) or -12 (a record larger
 * than data_file_size). */
typedef struct clyo_merge_result {
    uint64_t n_live, n_reencoded, hint_bytes;
    uint32_t n_out_files, _pad;
} clyo_merge_result;
int clyo_merge(const uint8_t* const* bases, const uint32_t* tuple_file, const clyo_tuple* tuples,
               uint64_t ntuples, const uint8_t* live, uint64_t data_file_size,
               uint8_t* out, uint32_t out_max_files, uint64_t* out_len,
               uint8_t* hint, uint64_t hint_cap, clyo_merge_result* res);

/* ---- CPU baselines for bench.py (cpu_baseline leg) ----------------------- */

/* "ref-faithful": scans one on-disk file reproducing the reference's I/O
 * pattern per ReadLogRecord: fstat, then open+fstat+mmap(whole file)+copy+
 * munmap+close for the header read and again for the key/value read
 * (driver/mmap.go:25-32, driver/fileIO.go:35-41, data/dataFile.go:64-111).
 * Stops after max_records (0 = no limit).  Returns records scanned, or -1. */
int64_t clyo_scan_path_faithful(const char* path, uint32_t fid, uint64_t max_records,
                                int64_t* end_offset, int32_t* status);

/* "ref-algorithm": files in memory, each scanned by clyo_scan_file, files
 * distributed over nthreads threads; tuples are produced (into per-thread
 * scratch) and counted.  Returns total records. */
uint64_t clyo_scan_files_mt(const uint8_t* const* bases, const uint64_t* lens,
                            const uint32_t* fids, int nfiles, int nthreads);

/* db.loadIndex (db.go:487-651) for the String and ListMeta types, one thread:
 * tx buffering by txId (:578, :604-626), last-writer-wins Put/Del (:511-554),
 * WriteOff of the last file (:633-635) and the TTL pass (:638-649, keys whose
 * expiration <= now_ns are deleted).  Returns 0, a scan error status, or
 * CLYO_LI_UNSUPPORTED for a Hash/List/Set record. */
enum { CLYO_LI_UNSUPPORTED = -20 };
typedef struct clyo_load_result {
    uint64_t records, applied, str_keys, listmeta_keys, expired, with_ttl, tx_pending;
    int64_t  write_off;
    int32_t  status, _pad;
} clyo_load_result;
int clyo_load_index(const uint8_t* const* bases, const uint64_t* lens, const uint32_t* fids, int nfiles,
                    int64_t now_ns, clyo_load_result* r);

#ifdef __cplusplus
}
#endif
#endif
