// Host-side BSON element walk for the persisted client results (no GPU).
//
// The reference persists every ClientResult as one BSON document in GridFS,
// `self._gridfs.put(bson.encode(result.dict()))` (client_daos.py:73), and reads
// it back with `ClientResult.parse_obj(bson.decode(results_file.read()))`
// (client_daos.py:142).  bson.decode copies the NPZ blob out of the document
// into a fresh bytes object.  fa_bson_elements only locates each element of one
// document level, so the host mirror (fedlesscan_amd/bsondoc.py) hands the blob
// on as a view into the GridFS bytes and the ingest packs it straight into
// pinned staging (fa_npz_index + fa_pack).
//
// Format: bsonspec.org 1.1, little-endian.  document = int32 total_len,
// element*, 0x00; element = type byte, cstring name, value.  Every length is
// checked against the enclosing document before it is used.
#include <cstdint>
#include <cstring>

#include "fedavg_hip.h"

namespace {

struct Walk {
    const uint8_t* b;
    int64_t end;  // one past the document's trailing 0x00

    bool i32(int64_t off, int32_t* v) const {
        if (off < 0 || off + 4 > end) return false;
        std::memcpy(v, b + off, 4);
        return true;
    }
    // offset of the NUL ending the cstring at off, or -1 (must end before `lim`)
    int64_t cstr(int64_t off, int64_t lim) const {
        if (off < 0 || off >= lim) return -1;
        const void* z = std::memchr(b + off, 0, (size_t)(lim - off));
        return z ? (int64_t)((const uint8_t*)z - b) : -1;
    }
    // BSON string: int32 length (bytes incl. the NUL) then the bytes
    bool str(int64_t p, int64_t lim, int64_t* voff, int64_t* vlen, int64_t* next) const {
        int32_t L;
        if (!i32(p, &L) || L < 1 || p + 4 + (int64_t)L > lim || b[p + 4 + L - 1] != 0) return false;
        *voff = p + 4;
        *vlen = L - 1;
        *next = p + 4 + L;
        return true;
    }
};

}  // namespace

extern "C" int64_t fa_bson_elements(const uint8_t* buf, int64_t buf_len, int64_t doc_off, uint8_t* types,
                                    int64_t* name_offs, int32_t* name_lens, int64_t* val_offs,
                                    int64_t* val_lens, uint8_t* subtypes, int64_t max_elems) {
    if (!buf || buf_len < 5 || doc_off < 0 || doc_off > buf_len - 5 || max_elems < 0) return FA_BSON_MALFORMED;
    int32_t total;
    std::memcpy(&total, buf + doc_off, 4);
    if (total < 5 || (int64_t)total > buf_len - doc_off) return FA_BSON_MALFORMED;
    const Walk w{buf, doc_off + total};
    const int64_t last = w.end - 1;  // the terminating 0x00
    if (buf[last] != 0) return FA_BSON_MALFORMED;
    int64_t p = doc_off + 4, n = 0;
    while (p < last) {
        const uint8_t t = buf[p++];
        const int64_t zn = w.cstr(p, last);
        if (zn < 0) return FA_BSON_MALFORMED;
        const int64_t name_off = p, name_len = zn - p;
        p = zn + 1;
        int64_t voff = p, vlen = 0, next = p;
        uint8_t sub = 0;
        switch (t) {
            case 0x01: case 0x09: case 0x11: case 0x12:  // double, UTC datetime, timestamp, int64
                vlen = 8; next = p + 8; break;
            case 0x10: vlen = 4; next = p + 4; break;    // int32
            case 0x07: vlen = 12; next = p + 12; break;  // ObjectId
            case 0x13: vlen = 16; next = p + 16; break;  // decimal128
            case 0x08:                                   // bool: exactly 0 or 1
                if (p >= last || buf[p] > 1) return FA_BSON_MALFORMED;
                vlen = 1; next = p + 1; break;
            case 0x06: case 0x0A: case 0x7F: case 0xFF:  // undefined, null, max key, min key
                break;
            case 0x02: case 0x0D: case 0x0E:             // string, JS code, symbol
                if (!w.str(p, last, &voff, &vlen, &next)) return FA_BSON_MALFORMED;
                break;
            case 0x03: case 0x04: {                      // embedded document / array
                int32_t L;
                if (!w.i32(p, &L) || L < 5 || p + (int64_t)L > last || buf[p + L - 1] != 0)
                    return FA_BSON_MALFORMED;
                vlen = L; next = p + L; break;
            }
            case 0x05: {                                 // binary: int32 len, subtype, bytes
                int32_t L;
                if (!w.i32(p, &L) || L < 0 || p + 5 + (int64_t)L > last) return FA_BSON_MALFORMED;
                sub = buf[p + 4];
                voff = p + 5; vlen = L; next = p + 5 + L;
                if (sub == 0x02) {                       // old binary: repeats the length inside
                    int32_t inner;
                    if (L < 4 || !w.i32(voff, &inner) || inner != L - 4) return FA_BSON_MALFORMED;
                    voff += 4; vlen -= 4;
                }
                break;
            }
            case 0x0B: {                                 // regex: pattern cstring, options cstring
                const int64_t z1 = w.cstr(p, last);
                const int64_t z2 = z1 < 0 ? -1 : w.cstr(z1 + 1, last);
                if (z2 < 0) return FA_BSON_MALFORMED;
                vlen = z2 + 1 - p; next = z2 + 1; break;
            }
            case 0x0C: {                                 // DBPointer: string + 12-byte ObjectId
                int64_t so, sl, sn;
                if (!w.str(p, last, &so, &sl, &sn)) return FA_BSON_MALFORMED;
                vlen = sn + 12 - p; next = sn + 12; break;
            }
            case 0x0F: {                                 // code with scope: int32 total, string, document
                int32_t L;
                if (!w.i32(p, &L) || L < 14 || p + (int64_t)L > last) return FA_BSON_MALFORMED;
                vlen = L; next = p + L; break;
            }
            default:
                return FA_BSON_UNSUPPORTED;
        }
        if (next > last) return FA_BSON_MALFORMED;
        if (n < max_elems) {
            if (types) types[n] = t;
            if (name_offs) name_offs[n] = name_off;
            if (name_lens) name_lens[n] = (int32_t)name_len;
            if (val_offs) val_offs[n] = voff;
            if (val_lens) val_lens[n] = vlen;
            if (subtypes) subtypes[n] = sub;
        }
        ++n;
        p = next;
    }
    return p == last ? n : FA_BSON_MALFORMED;
}
