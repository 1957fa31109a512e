// Host-side BSON element walk for the persisted client results (no GPU).
//
// The reference persists every ClientResult as one BSON document in GridFS,
// `self._gridfs.put(bson.encode(result.dict()))` (client_daos.py:73), and reads
// it back with `ClientResult.parse_obj(bson.decode(results_file.read()))`
// (client_daos.py:142).  bson.decode copies the NPZ blob out of the document
// into a fresh bytes object.  fa_bson_elements (one document level) and
// fa_bson_walk (the whole tree, one call) only locate the elements, so the host
// mirror (fedlesscan_amd/bsondoc.py) hands the blob on as a view into the
// GridFS bytes and the ingest packs it straight into pinned staging
// (fa_npz_index + fa_pack).
//
// Format: bsonspec.org 1.1, little-endian.  document = int32 total_len,
// element*, 0x00; element = type byte, cstring name, value.  Every length is
// checked against the enclosing document before it is used.
#include <cstdint>
#include <cstring>
#include <climits>

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

// One document level: calls sink(t, name_off, name_len, val_off, val_len, sub)
// per element in order; returns the element count or a FA_BSON_* code.
template <class Sink>
int64_t walk_level(const uint8_t* buf, int64_t buf_len, int64_t doc_off, Sink&& sink) {
    if (!buf || buf_len < 5 || doc_off < 0 || doc_off > buf_len - 5) return FA_BSON_MALFORMED;
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
        const int64_t rc = sink(t, name_off, name_len, voff, vlen, sub);
        if (rc < 0) return rc;
        ++n;
        p = next;
    }
    return p == last ? n : FA_BSON_MALFORMED;
}

struct Out {
    uint8_t* types; int32_t* parents; int64_t* name_offs; int32_t* name_lens;
    int64_t* val_offs; int64_t* val_lens; uint8_t* subtypes; int64_t max;
    void put(int64_t k, uint8_t t, int32_t parent, int64_t no, int64_t nl, int64_t vo, int64_t vl, uint8_t sub) const {
        if (k >= max) return;
        if (types) types[k] = t;
        if (parents) parents[k] = parent;
        if (name_offs) name_offs[k] = no;
        if (name_lens) name_lens[k] = (int32_t)nl;
        if (val_offs) val_offs[k] = vo;
        if (val_lens) val_lens[k] = vl;
        if (subtypes) subtypes[k] = sub;
    }
};

constexpr int kMaxDepth = 100;

// pre-order: each element, then (for documents and arrays) its subtree
int64_t walk_tree(const uint8_t* buf, int64_t buf_len, int64_t doc_off, int32_t parent, int depth,
                  const Out& out, int64_t* count) {
    if (depth > kMaxDepth) return FA_BSON_MALFORMED;
    return walk_level(buf, buf_len, doc_off, [&](uint8_t t, int64_t no, int64_t nl, int64_t vo, int64_t vl,
                                                 uint8_t sub) -> int64_t {
        const int64_t me = (*count)++;
        if (me > INT32_MAX) return FA_BSON_MALFORMED;
        out.put(me, t, parent, no, nl, vo, vl, sub);
        if (t == 0x03 || t == 0x04) return walk_tree(buf, buf_len, vo, (int32_t)me, depth + 1, out, count);
        return 0;
    });
}

}  // namespace

extern "C" int64_t fa_bson_elements(const uint8_t* buf, int64_t buf_len, int64_t doc_off, uint8_t* types,
                                    int64_t* name_offs, int32_t* name_lens, int64_t* val_offs,
                                    int64_t* val_lens, uint8_t* subtypes, int64_t max_elems) {
    if (max_elems < 0) return FA_BSON_MALFORMED;
    const Out out{types, nullptr, name_offs, name_lens, val_offs, val_lens, subtypes, max_elems};
    int64_t k = 0;
    return walk_level(buf, buf_len, doc_off, [&](uint8_t t, int64_t no, int64_t nl, int64_t vo, int64_t vl,
                                                 uint8_t sub) -> int64_t {
        out.put(k++, t, -1, no, nl, vo, vl, sub);
        return 0;
    });
}

extern "C" int64_t fa_bson_walk(const uint8_t* buf, int64_t buf_len, int64_t doc_off, uint8_t* types,
                                int32_t* parents, int64_t* name_offs, int32_t* name_lens, int64_t* val_offs,
                                int64_t* val_lens, uint8_t* subtypes, int64_t max_elems) {
    if (max_elems < 0) return FA_BSON_MALFORMED;
    const Out out{types, parents, name_offs, name_lens, val_offs, val_lens, subtypes, max_elems};
    int64_t count = 0;
    const int64_t rc = walk_tree(buf, buf_len, doc_off, -1, 0, out, &count);
    return rc < 0 ? rc : count;
}
