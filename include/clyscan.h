/*
 * clyscan.h — C-ABI drop-in boundary for CouloyDB's full-data-file log-record
 * scan, executed on an AMD Instinct MI355X (gfx950).
 *
 * Reference interface replaced (paths relative to the CouloyDB tree):
 *   func (df *DataFile) ReadLogRecord(offset int64) (*LogRecord, int64, error)
 *       data/dataFile.go:64-111, called in a loop "offset += size until io.EOF"
 *       by db.loadIndex          db.go:582-637   (index rebuild at open)
 *          db.merge              merge.go:90-143 (compaction)
 *          db.loadIndexFromHintFile merge.go:257-287 (hint file)
 *   DecodeLogRecordHeader        data/logRecord.go:86-114
 *   GetLogRecordCRC (+ compare)  data/logRecord.go:136-146, data/dataFile.go:105-109
 *   parseLogRecordKey            db.go:706-710   (tx_id / txid_len in cly_tuple)
 *
 * One call scans whole files: for every file it returns exactly the sequence of
 * records that repeated ReadLogRecord(offset) calls return from offset 0, and the
 * way that loop stops (io.EOF variants, ErrInvalidCRC, or the reference's panics
 * mapped to error codes).  Plain C types only; no HIP/torch types cross the ABI.
 *
 * Threading: a cly_ctx owns one GPU's scratch memory and one HIP stream; calls on
 * one context must be serialised by the caller (the reference scans on a single
 * goroutine during open, db.go:104-112).  Use one context per GPU.
 * Ownership: every buffer is caller-owned; nothing is retained after return.
 */
#ifndef CLYSCAN_H
#define CLYSCAN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- per-file terminal status (cly_file_result.status) --------------------
 * >= 0 : the reference loop sees io.EOF and stops cleanly (db.go:594-595).
 * <  0 : the reference returns an error (or panics) out of loadIndex/merge.   */
#define CLY_END_EOF      0   /* <=4 bytes left: DecodeLogRecordHeader -> nil   (logRecord.go:87-89, dataFile.go:82-84) */
#define CLY_END_ZERO     1   /* crc==0 && KeySize==0 && ValueSize==0            (dataFile.go:85-87)                   */
#define CLY_END_TORN     2   /* key/value run past EOF: mmap ReadAt short read -> io.EOF (dataFile.go:94-98)          */
#define CLY_ERR_CRC     -1   /* public.ErrInvalidCRC                            (dataFile.go:105-109)                 */
#define CLY_ERR_TRUNC5  -2   /* exactly 5 bytes left: buf[5] index panic        (logRecord.go:94)                     */
#define CLY_ERR_VARINT  -3   /* varint overflow drives a slice index negative, or headerSize<4 at the CRC slice (panics) */
#define CLY_ERR_OFFSET  -4   /* key/value read at a negative offset: "mmap: invalid ReadAt offset" (non-EOF error)    */

/* ---- API return codes ---------------------------------------------------- */
#define CLY_OK              0
#define CLY_ERR_CAPACITY  -10  /* out_cap too small for the records found            */
#define CLY_ERR_DEVICE    -11  /* HIP runtime error                                  */
#define CLY_ERR_ARG       -12  /* bad argument (null pointer, file >= 2^47 B, ...)   */
#define CLY_ERR_NOREPAIR  -13  /* speculation repair did not converge (never seen)   */

/* A data file (`%09d.cly`, hint-index or merge-finished file).  For cly_scan the
 * base is host memory (typically an mmap of the file); for cly_scan_device it is
 * device memory (HBM) that holds the file's bytes.  len < 2^47 (files are
 * walked in parts of 2 GiB, each seeing up to 4 GiB - 128 KiB from its start:
 * a record of over 2 GiB that crosses a part's end beyond that view fails the
 * call with CLY_ERR_ARG).                                                      */
typedef struct cly_file {
    const uint8_t* base;
    uint64_t       len;
    uint32_t       fid;       /* data.LogPos.Fid of records in this file        */
    uint32_t       _pad;
} cly_file;

/* One decoded record = one successful ReadLogRecord call (48 bytes, file order).
 * Key bytes live at base[offset+header_size .. offset+header_size+key_size);
 * the realKey of parseLogRecordKey starts txid_len bytes later.                */
typedef struct cly_tuple {
    int64_t  offset;          /* LogPos.Offset (db.go:601)                      */
    int64_t  expiration;      /* LogRecord.Expiration                           */
    int64_t  tx_id;           /* parseLogRecordKey txId (db.go:707); 0 if none  */
    uint32_t fid;             /* LogPos.Fid                                     */
    uint32_t size;            /* recordSize returned by ReadLogRecord           */
    uint32_t key_size;        /* LogRecordHeader.KeySize                        */
    uint32_t value_size;      /* LogRecordHeader.ValueSize                      */
    uint8_t  type;            /* LogRecord.Type  (0 Normal .. 4 TxnBegin)        */
    uint8_t  data_type;       /* LogRecord.DataType (0 String .. 4 Set)          */
    uint8_t  header_size;     /* headerSize from DecodeLogRecordHeader          */
    uint8_t  txid_len;        /* bytes of the txId varint; 0xFF = Varint overflow
                                 (parseLogRecordKey would panic)                 */
    uint32_t crc;             /* stored (and verified) CRC32-IEEE               */
} cly_tuple;

typedef struct cly_file_result {
    uint64_t n_records;       /* tuples emitted for this file                   */
    int64_t  end_offset;      /* EOF statuses: final offset (= activityFile.WriteOff,
                                 db.go:634-636); errors: offset of the failing record */
    int32_t  status;          /* CLY_END_* / CLY_ERR_*                           */
    int32_t  _pad;
} cly_file_result;

/* Timing of the last call (device work only; filled when requested).          */
typedef struct cly_stats {
    double   scan_ms;         /* decode+CRC kernel(s), HIP events; without the
                                 per-kernel markers (a debug option: each costs a
                                 ~5-us gap) this includes the link and the
                                 per-file result kernel                          */
    double   resolve_ms;      /* chain resolution (host-driven repair rounds;
                                 with the markers also the link and the per-file
                                 result kernel)                                  */
    double   total_ms;        /* whole device pipeline incl. repair passes     */
    uint32_t passes;          /* 1 = speculation verified first time           */
    uint32_t n_chunks;
    uint64_t bytes;           /* input bytes scanned                           */
    uint64_t records;         /* tuples emitted over all files                 */
} cly_stats;

typedef struct cly_ctx cly_ctx;

int  cly_ctx_create(int device, cly_ctx** out);
void cly_ctx_destroy(cly_ctx* ctx);
/* The clock of loadIndex's TTL sweep (db.go:639-651: a String key whose
 * winning put has Expiration != 0 and not after time.Now() is db.Del'd):
 * now_ns = UnixNano; 0 (the default) = the wall clock at each index call.    */
void cly_ctx_set_clock(cly_ctx* ctx, int64_t now_ns);

/* Upper bound on tuples for files whose records are >= 9 bytes (every record
 * the reference writer produces is).  Exotic records shorter than that make
 * cly_scan* return CLY_ERR_CAPACITY with the exact need in *needed.            */
uint64_t cly_scan_capacity(const cly_file* files, int nfiles);

/* Host-memory entry (the cgo path): copies the files to HBM, scans them, and
 * copies tuples back.  file_first[i] = index in `out` of file i's first tuple. */
int cly_scan(cly_ctx* ctx, const cly_file* files, int nfiles,
             cly_tuple* out, uint64_t out_cap,
             uint64_t* file_first, cly_file_result* res,
             uint64_t* needed, cly_stats* stats);

/* Device-resident entry: files[i].base are device pointers, d_out is device
 * memory; file_first/res/needed/stats are host memory.  `stream` is a
 * hipStream_t passed as void* (NULL = the context's own stream).               */
int cly_scan_device(cly_ctx* ctx, const cly_file* files, int nfiles,
                    cly_tuple* d_out, uint64_t out_cap,
                    uint64_t* file_first, cly_file_result* res,
                    uint64_t* needed, cly_stats* stats, void* stream);

/* ---- merge rewrite (db.merge, merge.go:90-143) ----------------------------
 * For every tuple of a scan whose live byte is set (the caller's index still
 * points at (fid, offset): merge.go:104-132), re-append the record to the merge
 * DB with Key = encodeKeyWithTxId(realKey, NO_TX_ID) (merge.go:129,
 * batch.go:120-127) through appendLogRecord (db.go:368-413: EncodeLogRecord, a
 * new file when WriteOff+size > data_file_size; the merge DB's first file is
 * fid 0), and write the hint record {realKey, EncodeLogRecordPos(pos)}
 * (merge.go:135, data/dataFile.go:114-121) to the hint-index file.
 * Output data file k (fid k) is at out + k*out_stride, out_stride =
 * data_file_size rounded up to 4 KiB; out_file_len[k] its length.  The
 * merge-finished file (merge.go:150-163) is the caller's: one record.
 * Returns CLY_OK; the scan's error status when a file's scan failed (the
 * reference's merge returns it); CLY_ERR_VARINT when a tuple's txId varint
 * overflowed (parseLogRecordKey panics); CLY_ERR_CAPACITY when out_max_files or
 * hint_cap is too small (mres holds the need; out/hint may be NULL to query);
 * CLY_ERR_ARG for a record larger than data_file_size.                         */
typedef struct cly_merge_result {
    uint64_t n_live;          /* records rewritten (= hint records)             */
    uint64_t n_reencoded;     /* live records whose bytes change (tx records)   */
    uint64_t hint_bytes;      /* length of the hint-index file                  */
    uint64_t out_stride;      /* distance between output files in `out`        */
    uint32_t n_out_files;     /* merge data files, fids 0 .. n_out_files-1      */
    uint32_t _pad;
    double   merge_ms;        /* device time of the merge kernels (device entry) */
} cly_merge_result;

/* Device-resident entry: files[i].base, d_tuples, d_live, d_out, d_hint are
 * device memory; d_tuples/file_first/res as cly_scan_device returned them
 * (files' tuples back to back); d_live[i] is the live byte of d_tuples[i].     */
int cly_merge_device(cly_ctx* ctx, const cly_file* files, int nfiles,
                     const cly_tuple* d_tuples, const uint64_t* file_first, const cly_file_result* res,
                     const uint8_t* d_live, uint64_t data_file_size,
                     uint8_t* d_out, uint32_t out_max_files, uint64_t* out_file_len,
                     uint8_t* d_hint, uint64_t hint_cap, cly_merge_result* mres, void* stream);

/* Host-memory entry (the cgo path): scans the files on the device, then
 * merges; live[i] (n_live_bytes = number of records the scan returns, in scan
 * order) is the index's verdict for the i-th record.                           */
int cly_merge(cly_ctx* ctx, const cly_file* files, int nfiles,
              const uint8_t* live, uint64_t n_live_bytes, uint64_t data_file_size,
              uint8_t* out, uint32_t out_max_files, uint64_t* out_file_len,
              uint8_t* hint, uint64_t hint_cap, cly_merge_result* mres);

/* ---- hint-index load (db.loadIndexFromHintFile, merge.go:257-287) -------- */
/* data.LogPos decoded from a hint record's value (DecodeLogRecordPos,
 * data/logRecord.go:126-134).                                                   */
typedef struct cly_pos {
    int64_t  offset;          /* LogPos.Offset                                  */
    uint32_t fid;             /* LogPos.Fid = uint32(first varint)              */
    uint32_t _pad;
} cly_pos;

/* Device entry: d_pos[i] = DecodeLogRecordPos(value of d_tuples[i]) for the n
 * tuples of a hint-file scan (cly_scan_device over d_hint_file).  Returns
 * CLY_ERR_VARINT when a value's first varint overflows (the reference panics);
 * *first_bad = the first such index (n if none).                              */
int cly_hint_positions_device(cly_ctx* ctx, const uint8_t* d_hint_file, const cly_tuple* d_tuples,
                              uint64_t n, cly_pos* d_pos, uint64_t* first_bad, void* stream);

/* Host entry: scan a hint-index file (host memory) and decode every record's
 * position: out[i] (Key = the realKey), pos[i].  *n_out = records returned
 * (the loop's io.EOF end, or the records before a decode panic, with
 * CLY_ERR_VARINT); res = the scan's per-file result (ErrInvalidCRC etc.).      */
int cly_hint_scan(cly_ctx* ctx, const cly_file* hint_file, cly_tuple* out, cly_pos* pos, uint64_t cap,
                  uint64_t* n_out, cly_file_result* res);

/* ---- index rebuild (db.loadIndex, db.go:511-651) -------------------------
 * Per record of a scan (scan order = fid order, offsets within), the state of
 * the five indexes after the load: records without a txId are applied at
 * once, records with a txId at their txId's next TxnCommit marker (a
 * TxnRollback drops them, TxnBegin is ignored, no marker: never applied); the
 * last applied record of a key decides (Put -> the index points at it,
 * Deleted -> the key is absent); a String key whose winning put has expired
 * (expiration set and <= the context clock, cly_ctx_set_clock) is dropped by
 * the TTL sweep (db.go:639-651).  Keys: String/ListMeta realKey; Hash
 * (key, field) = decodeFieldKey; List (key, seq.GobEncode()) = decodeListKey
 * with big.Float's gob re-encoding; Set (key, hashMemberKey) — updateIndex
 * decodes the stored key (txId varint included) of a record without a txId
 * and the realKey of a committed tx record (db.go:521-572, 600-620).
 * A hint file loaded before (loadIndexFromHintFile) is not part of this.     */
#define CLY_IX_DEAD 0         /* not the index's entry after the load         */
#define CLY_IX_LIVE 1         /* an index points here, and merge.go's lookup
                                 (merge.go:101-132) finds it: merge keeps it  */
#define CLY_IX_HOST 2         /* (no longer emitted: every data type is built
                                 on the device)                               */
#define CLY_IX_LOADONLY 3     /* an index points here, but merge.go decodes the
                                 realKey and looks up another key: a Hash/List/
                                 Set record without a txId; merge drops it    */
#define CLY_IX_EXPIRED 4      /* a String key's winning put, removed by the TTL
                                 sweep (db.Del: a tombstone goes to the active
                                 file); no index entry                        */
typedef struct cly_index_result {
    uint64_t n_live;          /* index entries (= records LIVE or LOADONLY)     */
    uint64_t n_applied;       /* records updateIndex sees                       */
    uint64_t n_host;          /* 0 (kept for layout)                            */
    uint64_t n_collisions;    /* sort-hash collisions: records whose key differs
                                 from the one before them in hash order
                                 (resolved exactly; informational)           */
    double   index_ms;        /* device time                                    */
    uint64_t n_loadonly;      /* records in state LOADONLY                      */
    uint64_t n_merge_panic;   /* Hash/List/Set records whose realKey decode
                                 panics in merge.go (a merge would fail)      */
} cly_index_result;

/* Device entry over a cly_scan_device result (tuples back to back): d_state
 * gets one byte per tuple.  The LIVE bytes are merge.go:104-132's liveness
 * (cly_merge_device's d_live takes d_state as is: it keeps state 1 only).
 * Returns the scan's error status if a file failed (loadIndex returns it),
 * CLY_ERR_VARINT if a txId varint overflowed or a Hash/List/Set key decode
 * that updateIndex applies panics (a slice bound out of range in Go).      */
int cly_index_device(cly_ctx* ctx, const cly_file* files, int nfiles,
                     const cly_tuple* d_tuples, const uint64_t* file_first, const cly_file_result* res,
                     uint8_t* d_state, cly_index_result* ir, void* stream);

/* Host-memory entry: scans the files (host memory) on the device, then the
 * index rebuild; state[i] for the i-th record in scan order, *n_out records. */
int cly_index(cly_ctx* ctx, const cly_file* files, int nfiles, uint8_t* state, uint64_t cap,
              uint64_t* n_out, cly_index_result* ir);

/* ---- batched append (the write path, db.appendLogRecord over a batch) ------
 * db.go:368-413 as db.Put (NO_TX_ID) and WriteBatch.Commit (batch.go:62-118)
 * issue it: Key = encodeKeyWithTxId(key, tx_id), EncodeLogRecord, a new file
 * when WriteOff+size > data_file_size, continuing the active file at
 * write_off; with `commit`, WriteBatch's marker {encodeKeyWithTxId(
 * TX_COMMIT_KEY, tx_id), TxnCommit} follows the records.  Output region k is
 * file active_fid+k at d_out + k*out_stride (region 0 holds the active file:
 * its bytes below write_off are kept); d_pos[i] = the LogPos of record i
 * (the marker's last).                                                        */
typedef struct cly_rec_in {   /* one record to append (device pointers), 40 B  */
    const uint8_t* key;
    const uint8_t* value;
    uint32_t key_len, value_len;
    int64_t  expiration;
    uint8_t  type, data_type, _pad[6];
} cly_rec_in;
typedef struct cly_append_result {
    uint64_t bytes;           /* bytes appended                                 */
    uint64_t out_stride;
    uint64_t final_write_off; /* activityFile.WriteOff afterwards               */
    uint32_t final_fid;       /* activityFile.FileId afterwards                 */
    uint32_t n_out_files;     /* regions touched (the active file + new files)  */
    double   append_ms;
} cly_append_result;
int cly_append_device(cly_ctx* ctx, const cly_rec_in* d_recs, uint64_t n, int64_t tx_id, int commit,
                      uint32_t active_fid, uint64_t write_off, uint64_t data_file_size,
                      uint8_t* d_out, uint32_t out_max_files, uint64_t* out_file_len, cly_pos* d_pos,
                      cly_append_result* ar, void* stream);
/* Host-memory entry (cgo): recs[i].key/value point to host memory; region k's
 * bytes come back at out + k*out_stride (region 0 from write_off on), the
 * positions in pos[].  out = NULL queries n_out_files and out_stride.        */
int cly_append(cly_ctx* ctx, const cly_rec_in* recs, uint64_t n, int64_t tx_id, int commit,
               uint32_t active_fid, uint64_t write_off, uint64_t data_file_size,
               uint8_t* out, uint32_t out_max_files, uint64_t* out_file_len, cly_pos* pos,
               cly_append_result* ar);

const char* cly_strerror(int code);

/* Library build identification (gfx target, kernel configuration).            */
const char* cly_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* CLYSCAN_H */
