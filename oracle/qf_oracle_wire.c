/*
 * qf_oracle_wire.c -- CPU restatement of the FEC packet framing,
 * src/fec/encoder.rs:18-152 (Packet::from_raw, Packet::from_block,
 * Packet::to_raw).
 *
 * TEST INFRASTRUCTURE ONLY (see qf_oracle.h): the checker for the library's
 * host framing (qf_packet_to_raw / qf_packet_from_raw) and the device framing
 * kernels (qf_frame_batch_dev / qf_parse_frames_dev).  Nothing in the product
 * path links it.
 *
 * Frame: <is_systematic u8> [<coeff_len u16 BE> <coeffs>] <payload>.
 * Each reference error string maps to its own return code, so a test can
 * tell which check fired (ORACLE_FR_* in qf_oracle.h).
 */
#include <string.h>

#include "qf_oracle.h"

/* encoder.rs:124-152 Packet::to_raw.  `has_coeffs` is the reference's
 * `self.coefficients.is_some()`; `has_data` is `self.data.is_some()` (when
 * absent the payload bytes of the buffer are left untouched but still
 * counted, encoder.rs:146-149). */
int oracle_packet_to_raw(int is_systematic, int has_coeffs, const uint8_t *coeffs,
                         uint32_t coeff_len, int has_data, const uint8_t *data, uint32_t len,
                         uint8_t *buffer, size_t buffer_len, size_t *written) {
    size_t required_len = (size_t)len + 1;                 /* encoder.rs:125 */
    if (has_coeffs) required_len += 2 + (size_t)coeff_len; /* encoder.rs:126-128 */
    if (buffer_len < required_len) return ORACLE_FR_BUFFER_TOO_SHORT; /* encoder.rs:129-131 */
    size_t offset = 0;
    buffer[offset] = is_systematic ? 1 : 0; /* encoder.rs:134 */
    offset += 1;
    if (has_coeffs) {
        const uint16_t cl = (uint16_t)coeff_len; /* `as u16` truncates (encoder.rs:138) */
        buffer[offset] = (uint8_t)(cl >> 8);
        buffer[offset + 1] = (uint8_t)(cl & 0xFF);
        offset += 2;
        memcpy(buffer + offset, coeffs, coeff_len); /* encoder.rs:141-143 */
        offset += coeff_len;
    }
    if (has_data) memcpy(buffer + offset, data, len); /* encoder.rs:146-148 */
    offset += len;
    *written = offset;
    return ORACLE_OK;
}

/* encoder.rs:18-68 Packet::from_raw.  `block_size` is the pool block size of
 * opt_manager.alloc_block() (optimize.rs:135-142, default 4096).  On success:
 * *is_systematic, *coeff_len, *coeff_off (offset of the coefficients in raw),
 * *payload_off and *len (the payload is raw[payload_off .. payload_off+len)). */
int oracle_packet_from_raw(const uint8_t *raw, size_t raw_len, size_t block_size,
                           int *is_systematic, uint32_t *coeff_len, size_t *coeff_off,
                           size_t *payload_off, size_t *len) {
    if (raw_len == 0) return ORACLE_FR_EMPTY; /* encoder.rs:23-26 */
    const int sys = raw[0] == 1;              /* encoder.rs:28 */
    size_t offset = 1;
    uint32_t cl = 0;
    size_t coff = 0, poff;
    if (!sys) {
        if (raw_len < 3) return ORACLE_FR_NO_COEFF_LEN; /* encoder.rs:32-35 */
        cl = ((uint32_t)raw[offset] << 8) | raw[offset + 1]; /* encoder.rs:36-37 */
        offset += 2;
        if (raw_len < offset + cl) return ORACLE_FR_COEFF_TRUNCATED; /* encoder.rs:40-43 */
        /* coeff_block[..coeff_len] indexes a pool block: a panic when the
         * coefficient vector is longer than the block (encoder.rs:44-45) */
        if (cl > block_size) return ORACLE_FR_PANIC;
        coff = offset;
        poff = offset + cl;
    } else {
        poff = offset;
    }
    const size_t plen = raw_len - poff; /* encoder.rs:51 */
    if (block_size < plen) return ORACLE_FR_POOL_TOO_SMALL; /* encoder.rs:52-56 */
    *is_systematic = sys;
    *coeff_len = cl;
    *coeff_off = coff;
    *payload_off = poff;
    *len = plen;
    return ORACLE_OK;
}

/* encoder.rs:72-121 Packet::from_block.  The block (block_len bytes, `len`
 * of them valid) is rewritten in place: the payload is moved to the front
 * (copy_within, encoder.rs:107-110), bytes after it keep their old values.
 * The coefficients are copied out to coeffs_out (a second pool block of
 * block_len bytes, encoder.rs:100-101). */
int oracle_packet_from_block(uint8_t *block, size_t block_len, size_t len, int *is_systematic,
                             uint8_t *coeffs_out, uint32_t *coeff_len, size_t *payload_len) {
    if (len == 0 || len > block_len) return ORACLE_FR_INVALID_LEN; /* encoder.rs:78-82 */
    const int sys = block[0] == 1;                                  /* encoder.rs:84 */
    size_t offset = 1;
    uint32_t cl = 0;
    size_t poff;
    if (!sys) {
        if (len < 3) return ORACLE_FR_NO_COEFF_LEN; /* encoder.rs:88-92 */
        cl = ((uint32_t)block[offset] << 8) | block[offset + 1]; /* encoder.rs:93 */
        offset += 2;
        if (len < offset + cl) return ORACLE_FR_COEFF_TRUNCATED; /* encoder.rs:95-99 */
        if (cl > block_len) return ORACLE_FR_PANIC;              /* coeff_block[..coeff_len] */
        if (coeffs_out) memcpy(coeffs_out, block + offset, cl);  /* encoder.rs:100-101 */
        poff = offset + cl;
    } else {
        poff = offset;
    }
    const size_t plen = len - poff;                      /* encoder.rs:107 */
    if (poff > 0) memmove(block, block + poff, len - poff); /* encoder.rs:108-110 */
    *is_systematic = sys;
    *coeff_len = cl;
    *payload_len = plen;
    return ORACLE_OK;
}
