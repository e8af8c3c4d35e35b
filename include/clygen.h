/*
 * clygen.h — synthetic CouloyDB data-file writer on the GPU (bench/test input).
 *
 * Restates the reference's write side so that device-resident inputs of the
 * BASELINE.json configurations can be produced at HBM speed:
 *   EncodeLogRecord            data/logRecord.go:57-84   (header varints + CRC32)
 *   encodeKeyWithTxId          batch.go:120-127          (key = varint(txId) || key)
 *   appendLogRecord rotation   db.go:376-385             (new file when full)
 *   bytex.GetTestKey / RandomBytes  public/utils/bytex/bytex.go:13-23
 * Not part of the scan ABI (include/clyscan.h).
 */
#ifndef CLYGEN_H
#define CLYGEN_H
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

/* value_mode */
#define CLYGEN_VALUE_RANDOM   0   /* splitmix64 bytes                               */
#define CLYGEN_VALUE_KEYZERO  1   /* key digits then zero bytes (TestDB_Reboot)      */
#define CLYGEN_VALUE_ALNUM    2   /* charset bytes (bytex.RandomBytes)              */

/* One record to write: key = varint(tx_id) || "%09d"(key_index).  32 bytes.  */
typedef struct cly_gen_rec {
    uint64_t dst;          /* byte offset of the record in the device buffer    */
    uint32_t key_index;
    uint32_t value_len;
    int64_t  tx_id;
    uint8_t  type, dtype, value_mode, _pad;
    int32_t  _pad2;
} cly_gen_rec;

/* Encoded size of such a record (expiration 0). */
uint64_t cly_gen_record_size(int64_t tx_id, uint32_t value_len);

/* Lay records out into data files the way appendLogRecord does: a record
 * goes to a new file when WriteOff+size > data_file_size.  Files are placed in
 * the device buffer at offsets aligned to `align`.  Fills recs[i].dst and
 * file_len[0..*nfiles).  Returns total device bytes needed.                  */
uint64_t cly_gen_layout(cly_gen_rec* recs, uint64_t nrecs, uint64_t data_file_size,
                        uint64_t align, uint64_t* file_off, uint64_t* file_len,
                        uint32_t max_files, uint32_t* nfiles);

/* Encode records into device memory d_buf (one wavefront per record).
 * d_recs: device array of nrecs cly_gen_rec.  Synchronous.  Returns 0 / <0. */
int cly_gen_encode(uint8_t* d_buf, const cly_gen_rec* d_recs, uint64_t nrecs, uint64_t seed);

#ifdef __cplusplus
}
#endif
#endif
