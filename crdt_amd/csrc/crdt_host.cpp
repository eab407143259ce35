// crdt_host.cpp — native host ingest for the MapCrdt merge path (include/crdt_host.h).
//
// The device kernels (crdt_merge.hip) consume integer columns; this file turns the
// reference's wire format into them without a per-record trip through Python:
//   * crdt_keys      — key interning (LinkedHashMap order ids, map_crdt.dart:10)
//   * crdt_json_decode — CrdtJson.decode (crdt_json.dart:19-37) + Record.fromJson
//                      (record.dart:21-26) + Hlc.parse (hlc.dart:39-46) for the format
//                      CrdtJson.encode / Hlc.toString write (crdt_json.dart:8-17,
//                      hlc.dart:101-104); everything else is CRDT_HOST_FALLBACK.
//   * crdt_hlc_format  — Hlc.toString for a batch of clocks.
//   * crdt_json_encode — the export half of sync: CrdtJson.encode (crdt_json.dart:8-17) of a
//                      recordMap (map_crdt.dart:42-45) with Record.toJson (record.dart:28-31)
//                      and Hlc.toJson = toString (hlc.dart:101-104, 122); value texts come
//                      from the caller (crdt_json_canonical tells which raw input spans can
//                      be reused verbatim, crdt_json_split cuts one dumped array into values).
// Built with g++ -O3 (no GPU code).  Parity: tests/test_host_ingest.py compares every
// column with the Python restatement (crdt_amd/crdt_json.py, crdt_amd/hlc.py).
#include "crdt_host.h"

#include <stdint.h>
#include <string.h>

#include <stdlib.h>
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <functional>
#include <new>
#include <thread>
#include <string>
#include <string_view>
#include <unordered_set>
#include <unordered_map>
#include <vector>

namespace {

constexpr int kShift = 16;                        // hlc.dart:3
constexpr int64_t kMaxMs = 8640000000000000ll;    // DateTime range (ms)

inline uint64_t hash_bytes(const char* p, uint64_t n) {
    uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xff51afd7ed558ccdull);
    uint64_t i = 0;
    for (; i + 8 <= n; i += 8) {
        uint64_t w;
        memcpy(&w, p + i, 8);
        h = (h ^ w) * 0x100000001b3ull;
        h ^= h >> 29;
    }
    uint64_t t = 0;
    for (uint64_t k = 0; i + k < n; ++k) t |= (uint64_t)(uint8_t)p[i + k] << (8 * k);
    h = (h ^ t) * 0xc4ceb9fe1a85ec53ull;
    h ^= h >> 32;
    return h ? h : 1;
}

// Days since 1970-01-01 of a proleptic Gregorian date (any int month/day offsets).
inline int64_t days_from_civil(int64_t y, int64_t m, int64_t d) {
    y -= m <= 2;
    const int64_t era = (y >= 0 ? y : y - 399) / 400;
    const int64_t yoe = y - era * 400;
    const int64_t doy = (153 * ((m + 9) % 12) + 2) / 5 + d - 1;
    return era * 146097 + yoe * 365 + yoe / 4 - yoe / 100 + doy - 719468;
}

inline void civil_from_days(int64_t z, int64_t* y, int64_t* m, int64_t* d) {
    z += 719468;
    const int64_t era = (z >= 0 ? z : z - 146096) / 146097;
    const int64_t doe = z - era * 146097;
    const int64_t yoe = (doe - doe / 1460 + doe / 36524 - doe / 146096) / 365;
    const int64_t doy = doe - (365 * yoe + yoe / 4 - yoe / 100);
    const int64_t mp = (5 * doy + 2) / 153;
    *m = mp < 10 ? mp + 3 : mp - 9;
    *d = doy - (153 * mp + 2) / 5 + 1;
    *y = yoe + era * 400 + (*m <= 2);
}

inline int64_t floordiv(int64_t a, int64_t b) { return a / b - ((a % b != 0) && ((a < 0) != (b < 0))); }

inline int digit(char c) { return (c >= '0' && c <= '9') ? c - '0' : -1; }
inline int hexval(char c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

}  // namespace

// ------------------------------------------------------------------ key table
struct crdt_keys {
    std::vector<char> arena;
    std::vector<uint64_t> off{0};      // off[id] .. off[id + 1]
    std::vector<uint64_t> hash;        // per id (rebuilds)
    std::vector<uint64_t> slot;        // open addressing: (hash >> 32) << 32 | (id + 1), 0 = empty
    uint64_t mask = 0;

    uint64_t size() const { return hash.size(); }

    void rebuild(uint64_t want) {
        uint64_t cap = 16;
        while (cap < want * 2) cap <<= 1;
        slot.assign(cap, 0);
        mask = cap - 1;
        for (uint64_t id = 0; id < hash.size(); ++id) place(hash[id], (uint32_t)id);
    }

    void place(uint64_t h, uint32_t id) {
        uint64_t s = h & mask;
        while (slot[s]) s = (s + 1) & mask;
        slot[s] = (h & 0xFFFFFFFF00000000ull) | (uint64_t)(id + 1);
    }

    // the slot word carries the hash's high half: a probe touches the key bytes only on a match
    bool find(const char* p, uint64_t n, uint64_t h, uint32_t* id) const {
        if (slot.empty()) return false;
        const uint64_t hi = h & 0xFFFFFFFF00000000ull;
        for (uint64_t s = h & mask;; s = (s + 1) & mask) {
            const uint64_t v = slot[s];
            if (!v) return false;
            if ((v & 0xFFFFFFFF00000000ull) != hi) continue;
            const uint32_t i = (uint32_t)v - 1;
            if (off[i + 1] - off[i] == n && memcmp(arena.data() + off[i], p, n) == 0) {
                *id = i;
                return true;
            }
        }
    }

    void reserve(uint64_t more_keys, uint64_t more_bytes) {
        const uint64_t want = hash.size() + more_keys;
        if (want * 2 > slot.size()) rebuild(want);
        arena.reserve(arena.size() + more_bytes);
        off.reserve(want + 1);
        hash.reserve(want);
    }

    void prefetch(uint64_t h) const {
        if (!slot.empty()) __builtin_prefetch(slot.data() + (h & mask));
    }

    // One probe sequence: true with *id when present, else the key is added (next id), false.
    bool find_or_add(const char* p, uint64_t n, uint64_t h, uint32_t* id) {
        if ((hash.size() + 1) * 2 > slot.size()) rebuild(hash.size() + 1 > 8 ? (hash.size() + 1) * 2 : 16);
        const uint64_t hi = h & 0xFFFFFFFF00000000ull;
        uint64_t s = h & mask;
        for (;; s = (s + 1) & mask) {
            const uint64_t v = slot[s];
            if (!v) break;
            if ((v & 0xFFFFFFFF00000000ull) != hi) continue;
            const uint32_t i = (uint32_t)v - 1;
            if (off[i + 1] - off[i] == n && memcmp(arena.data() + off[i], p, n) == 0) {
                *id = i;
                return true;
            }
        }
        const uint32_t nid = (uint32_t)hash.size();
        arena.insert(arena.end(), p, p + n);
        off.push_back(arena.size());
        hash.push_back(h);
        slot[s] = hi | (uint64_t)(nid + 1);
        *id = nid;
        return false;
    }

    uint32_t add(const char* p, uint64_t n, uint64_t h) {
        if ((hash.size() + 1) * 2 > slot.size()) rebuild(hash.size() + 1 > 8 ? (hash.size() + 1) * 2 : 16);
        const uint32_t id = (uint32_t)hash.size();
        arena.insert(arena.end(), p, p + n);
        off.push_back(arena.size());
        hash.push_back(h);
        place(h, id);
        return id;
    }
};

// --------------------------------------------------------------- decode state
struct crdt_decoded {
    std::vector<uint32_t> key;
    std::vector<int64_t> lt;
    std::vector<uint32_t> node;
    std::vector<uint64_t> voff;
    std::vector<uint32_t> vlen;
    std::vector<std::string> nodes;
};

namespace {

struct Fallback {};
struct JsonError {};

struct Parser {
    const char* s;
    uint64_t n, i = 0;
    std::string tmp;

    void ws() {
        while (i < n && (s[i] == ' ' || s[i] == '\t' || s[i] == '\n' || s[i] == '\r')) ++i;
    }
    char peek() { return i < n ? s[i] : '\0'; }
    void expect(char c) {
        if (i >= n || s[i] != c) throw JsonError();
        ++i;
    }

    static void put_utf8(std::string& o, uint32_t cp) {
        if (cp < 0x80) {
            o += (char)cp;
        } else if (cp < 0x800) {
            o += (char)(0xC0 | (cp >> 6));
            o += (char)(0x80 | (cp & 0x3F));
        } else if (cp < 0x10000) {
            o += (char)(0xE0 | (cp >> 12));
            o += (char)(0x80 | ((cp >> 6) & 0x3F));
            o += (char)(0x80 | (cp & 0x3F));
        } else {
            o += (char)(0xF0 | (cp >> 18));
            o += (char)(0x80 | ((cp >> 12) & 0x3F));
            o += (char)(0x80 | ((cp >> 6) & 0x3F));
            o += (char)(0x80 | (cp & 0x3F));
        }
    }

    uint32_t hex4() {
        if (i + 4 > n) throw JsonError();
        uint32_t v = 0;
        for (int k = 0; k < 4; ++k) {
            const int h = hexval(s[i + k]);
            if (h < 0) throw JsonError();
            v = (v << 4) | (uint32_t)h;
        }
        i += 4;
        return v;
    }

    // A JSON string at s[i] ('"'): *p/*len = its UTF-8 text (in the input when it has no
    // escapes, else in tmp).  Lone UTF-16 surrogates have no UTF-8 form: fallback.
    void string(const char** p, uint64_t* len) {
        expect('"');
        const uint64_t b = i;
        while (i < n && s[i] != '"' && s[i] != '\\') {
            if ((uint8_t)s[i] < 0x20) throw JsonError();
            ++i;
        }
        if (i >= n) throw JsonError();
        if (s[i] == '"') {
            *p = s + b;
            *len = i - b;
            ++i;
            return;
        }
        tmp.assign(s + b, i - b);
        while (true) {
            if (i >= n) throw JsonError();
            const char c = s[i];
            if (c == '"') { ++i; break; }
            if ((uint8_t)c < 0x20) throw JsonError();
            if (c != '\\') { tmp += c; ++i; continue; }
            if (++i >= n) throw JsonError();
            const char e = s[i++];
            switch (e) {
                case '"': tmp += '"'; break;
                case '\\': tmp += '\\'; break;
                case '/': tmp += '/'; break;
                case 'b': tmp += '\b'; break;
                case 'f': tmp += '\f'; break;
                case 'n': tmp += '\n'; break;
                case 'r': tmp += '\r'; break;
                case 't': tmp += '\t'; break;
                case 'u': {
                    uint32_t cp = hex4();
                    if (cp >= 0xD800 && cp < 0xDC00) {
                        if (i + 6 <= n && s[i] == '\\' && s[i + 1] == 'u') {
                            i += 2;
                            const uint32_t lo = hex4();
                            if (lo < 0xDC00 || lo >= 0xE000) throw Fallback();
                            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
                        } else {
                            throw Fallback();
                        }
                    } else if (cp >= 0xDC00 && cp < 0xE000) {
                        throw Fallback();
                    }
                    put_utf8(tmp, cp);
                    break;
                }
                default: throw JsonError();
            }
        }
        *p = tmp.data();
        *len = tmp.size();
    }

    void skip_string() {
        expect('"');
        while (true) {
            if (i >= n) throw JsonError();
            const char c = s[i];
            if (c == '"') { ++i; return; }
            if ((uint8_t)c < 0x20) throw JsonError();
            if (c == '\\') {
                if (++i >= n) throw JsonError();
                const char e = s[i++];
                if (e == 'u') {
                    const uint32_t cp = hex4();
                    // values are re-read by the caller's JSON decoder; lone surrogates
                    // there are its business, but keep the fast path to well-formed text
                    if (cp >= 0xD800 && cp < 0xE000) throw Fallback();
                } else if (!strchr("\"\\/bfnrt", e)) {
                    throw JsonError();
                }
            } else {
                ++i;
            }
        }
    }

    void number() {
        const uint64_t b = i;
        if (peek() == '-') ++i;
        if (i >= n) throw JsonError();
        if (s[i] == '0') {
            ++i;
        } else if (s[i] >= '1' && s[i] <= '9') {
            while (i < n && digit(s[i]) >= 0) ++i;
        } else {
            // NaN / Infinity: Python's json accepts them, Dart's does not — let the caller decide
            if (s[i] == 'N' || s[i] == 'I') throw Fallback();
            throw JsonError();
        }
        if (peek() == '.') {
            ++i;
            if (digit(peek()) < 0) throw JsonError();
            while (i < n && digit(s[i]) >= 0) ++i;
        }
        if (peek() == 'e' || peek() == 'E') {
            ++i;
            if (peek() == '+' || peek() == '-') ++i;
            if (digit(peek()) < 0) throw JsonError();
            while (i < n && digit(s[i]) >= 0) ++i;
        }
        if (i == b) throw JsonError();
    }

    void literal(const char* w) {
        const uint64_t l = strlen(w);
        if (i + l > n || memcmp(s + i, w, l) != 0) throw JsonError();
        i += l;
    }

    void skip_value(int depth) {
        if (depth > 256) throw Fallback();
        ws();
        const char c = peek();
        if (c == '{') {
            ++i;
            ws();
            if (peek() == '}') { ++i; return; }
            while (true) {
                ws();
                skip_string();
                ws();
                expect(':');
                skip_value(depth + 1);
                ws();
                if (peek() == ',') { ++i; continue; }
                expect('}');
                return;
            }
        } else if (c == '[') {
            ++i;
            ws();
            if (peek() == ']') { ++i; return; }
            while (true) {
                skip_value(depth + 1);
                ws();
                if (peek() == ',') { ++i; continue; }
                expect(']');
                return;
            }
        } else if (c == '"') {
            skip_string();
        } else if (c == 't') {
            literal("true");
        } else if (c == 'f') {
            literal("false");
        } else if (c == 'n') {
            literal("null");
        } else if (c == 'N' || c == 'I') {
            throw Fallback();
        } else {
            number();
        }
    }
};

// Hlc.parse of the Hlc.toString form "YYYY-MM-DDTHH:MM:SS.mmmZ-XXXX-<node>" (hlc.dart:39-46:
// counterDash = indexOf('-', lastIndexOf(':')), nodeIdDash = indexOf('-', counterDash + 1),
// millis = DateTime.parse(..).millisecondsSinceEpoch, counter = int.parse(.., radix: 16)).
// The fast form needs its last ':' at 16 (no ':' in the node id).
bool parse_hlc(const char* t, uint64_t len, int64_t* lt, uint64_t* node_pos) {
    if (len < 30) return false;
    for (uint64_t k = 17; k < len; ++k)
        if (t[k] == ':') return false;
    static const char sep[24] = {0, 0, 0, 0, '-', 0, 0, '-', 0, 0, 'T', 0, 0, ':', 0, 0, ':', 0, 0, '.', 0, 0, 0, 'Z'};
    int64_t v[24];
    for (int k = 0; k < 24; ++k) {
        if (sep[k]) {
            if (t[k] != sep[k]) return false;
        } else {
            v[k] = digit(t[k]);
            if (v[k] < 0) return false;
        }
    }
    if (t[24] != '-' || t[29] != '-') return false;
    int64_t counter = 0;
    for (int k = 25; k < 29; ++k) {
        const int h = hexval(t[k]);
        if (h < 0) return false;
        counter = (counter << 4) | h;
    }
    int64_t year = v[0] * 1000 + v[1] * 100 + v[2] * 10 + v[3];
    const int64_t month = v[5] * 10 + v[6], day = v[8] * 10 + v[9];
    const int64_t hour = v[11] * 10 + v[12], minute = v[14] * 10 + v[15], second = v[17] * 10 + v[18];
    const int64_t milli = v[20] * 100 + v[21] * 10 + v[22];
    // DateTime.parse normalises out-of-range fields (as crdt_amd/hlc.py::millis_from_iso)
    int64_t mz = month - 1;
    year += floordiv(mz, 12);
    mz -= floordiv(mz, 12) * 12;
    const int64_t days = days_from_civil(year, mz + 1, 1) + day - 1;
    const int64_t ms = (((days * 24 + hour) * 60 + minute) * 60 + second) * 1000 + milli;
    if (ms > kMaxMs || ms < -kMaxMs) return false;
    // Hlc(millis, counter, nodeId): millis >= 2^48 would be microseconds — impossible here
    *lt = (int64_t)(((uint64_t)ms << kShift) + (uint64_t)counter);
    *node_pos = 30;
    return true;
}

// Open-addressing set of key ids met in one document -> their record index.
struct IdMap {
    std::vector<uint64_t> s;   // (id + 1) << 32 | record
    uint64_t mask = 0, used = 0;
    void init(uint64_t want) {
        uint64_t cap = 64;
        while (cap < want * 2) cap <<= 1;
        s.assign(cap, 0);
        mask = cap - 1;
        used = 0;
    }
    void prefetch(uint32_t id) const {
        __builtin_prefetch(s.data() + ((((uint64_t)id * 0x9E3779B97F4A7C15ull) >> 20) & mask));
    }
    // returns the record index of id, or inserts rec and returns UINT32_MAX
    uint32_t get_or_put(uint32_t id, uint32_t rec) {
        if ((used + 1) * 2 > s.size()) {
            std::vector<uint64_t> old;
            old.swap(s);
            init(old.size());
            for (uint64_t e : old)
                if (e) raw_put(e);
        }
        uint64_t h = ((uint64_t)id * 0x9E3779B97F4A7C15ull) >> 20;
        for (uint64_t k = h & mask;; k = (k + 1) & mask) {
            const uint64_t e = s[k];
            if (!e) {
                s[k] = ((uint64_t)(id + 1) << 32) | rec;
                ++used;
                return UINT32_MAX;
            }
            if ((e >> 32) == (uint64_t)id + 1) return (uint32_t)e;
        }
    }
    void raw_put(uint64_t e) {
        const uint32_t id = (uint32_t)(e >> 32) - 1;
        uint64_t h = ((uint64_t)id * 0x9E3779B97F4A7C15ull) >> 20;
        uint64_t k = h & mask;
        while (s[k]) k = (k + 1) & mask;
        s[k] = e;
        ++used;
    }
};

// One record `"<key>": {"hlc": <string>, "value": <any>, ...}` at p (after '{' or ','):
// the key (decoded UTF-8 into *key), Hlc.parse of hlc -> lt + node id span, value span.
struct RecordText {
    int64_t lt;
    const char* node;            // into the input (Hlc strings never need unescaping here: a
    uint64_t node_len;           // node id with an escape is copied into node_buf)
    uint64_t voff;
    uint32_t vlen;
};

void parse_record(Parser& p, const char* js, std::string& key, std::string& node_buf, RecordText& r) {
    const char* kp;
    uint64_t kl;
    p.string(&kp, &kl);
    key.assign(kp, kl);                               // p.tmp is reused below
    p.ws();
    p.expect(':');
    p.ws();
    // the record object: {"hlc": <string>, "value": <any>, ...}; a repeated field: last wins
    if (p.peek() != '{') throw Fallback();
    ++p.i;
    bool have_hlc = false;
    r.voff = 0;
    r.vlen = 0;
    p.ws();
    if (p.peek() == '}') {
        ++p.i;
    } else {
        while (true) {
            p.ws();
            const char* fp;
            uint64_t fl;
            p.string(&fp, &fl);
            const bool is_hlc = fl == 3 && memcmp(fp, "hlc", 3) == 0;
            const bool is_val = fl == 5 && memcmp(fp, "value", 5) == 0;
            p.ws();
            p.expect(':');
            p.ws();
            if (is_hlc) {
                if (p.peek() != '"') throw Fallback();
                const char* hp;
                uint64_t hl;
                p.string(&hp, &hl);
                uint64_t npos;
                if (!parse_hlc(hp, hl, &r.lt, &npos)) throw Fallback();
                node_buf.assign(hp + npos, hl - npos);
                have_hlc = true;
            } else if (is_val) {
                const uint64_t b = p.i;
                p.skip_value(1);
                const bool is_null = p.i - b == 4 && memcmp(js + b, "null", 4) == 0;
                if (p.i - b >= (1ull << 32)) throw Fallback();
                r.voff = is_null ? 0 : b;
                r.vlen = is_null ? 0 : (uint32_t)(p.i - b);
            } else {
                p.skip_value(1);
            }
            p.ws();
            if (p.peek() == ',') { ++p.i; continue; }
            p.expect('}');
            break;
        }
    }
    if (!have_hlc) throw Fallback();                  // Hlc.parse(null) throws
    r.node = node_buf.data();
    r.node_len = node_buf.size();
}

// Per-document builder of the output columns: node ids in first-seen order, key ids from the
// table (new keys appended in document order), a repeated key keeps its first position and
// its last record (jsonDecode into a LinkedHashMap).
struct Builder {
    crdt_keys* keys;
    crdt_decoded* d;
    uint64_t n0;                                      // table size before the document
    std::unordered_map<std::string, uint32_t> node_ix;
    IdMap seen;                                       // keys that existed before: id -> first record
    std::vector<uint32_t> first_new;                  // keys added by the document: first record
    const char* last_node = nullptr;                  // records of one changeset mostly share a node
    uint64_t last_len = 0;
    uint32_t last_nid = 0;

    Builder(crdt_keys* k, crdt_decoded* dd) : keys(k), d(dd), n0(k->size()) { seen.init(64); }

    uint32_t node_id(const char* np, uint64_t nl) {
        if (last_node && nl == last_len && memcmp(np, last_node, nl) == 0) return last_nid;
        const std::string node(np, nl);
        auto it = node_ix.find(node);
        uint32_t nid;
        if (it == node_ix.end()) {
            nid = (uint32_t)d->nodes.size();
            node_ix.emplace(node, nid);
            d->nodes.push_back(node);
        } else {
            nid = it->second;
        }
        last_node = d->nodes[nid].data();
        last_len = d->nodes[nid].size();
        last_nid = nid;
        return nid;
    }

    // id: the key's id when already known to exist (UINT32_MAX: look it up / add it now)
    void add(const char* kp, uint64_t kl, uint64_t h, uint32_t id, int64_t lt, uint32_t nid, uint64_t voff,
             uint32_t vlen) {
        const uint32_t rec = (uint32_t)d->key.size();
        uint32_t prev = UINT32_MAX;
        bool fresh = false;
        if (id == UINT32_MAX) {
            if (keys->size() >= 0xFFFFFFF0ull) throw Fallback();
            fresh = !keys->find_or_add(kp, kl, h, &id);
        }
        if (fresh) {
            first_new.push_back(rec);                   // id == n0 + first_new.size() - 1
        } else if (id >= n0) {
            prev = first_new[id - n0];                  // repeated in this document
        } else {
            prev = seen.get_or_put(id, rec);
        }
        if (prev != UINT32_MAX) {                     // repeated key: first position, last record
            d->lt[prev] = lt;
            d->node[prev] = nid;
            d->voff[prev] = voff;
            d->vlen[prev] = vlen;
        } else {
            d->key.push_back(id);
            d->lt.push_back(lt);
            d->node.push_back(nid);
            d->voff.push_back(voff);
            d->vlen.push_back(vlen);
        }
    }
};

void begin_object(Parser& p) {
    p.ws();
    p.expect('{');
    p.ws();
}

// After a record: true when another follows (p at its key), false at the closing '}'.
bool next_record(Parser& p) {
    p.ws();
    if (p.peek() == ',') {
        ++p.i;
        p.ws();
        return true;
    }
    p.expect('}');
    return false;
}

int decode_sequential(const char* js, uint64_t len, crdt_keys* keys, crdt_decoded* d) {
    Parser p{js, len, 0, std::string()};
    Builder bld(keys, d);
    const uint64_t est = len / 48 + 16;               // a record is >= ~48 bytes of JSON
    keys->reserve(est, len / 4);
    d->key.reserve(est); d->lt.reserve(est); d->node.reserve(est); d->voff.reserve(est); d->vlen.reserve(est);
    std::string key, node;
    RecordText r;
    begin_object(p);
    if (p.peek() == '}') {
        ++p.i;
    } else {
        do {
            parse_record(p, js, key, node, r);
            bld.add(key.data(), key.size(), hash_bytes(key.data(), key.size()), UINT32_MAX, r.lt,
                    bld.node_id(r.node, r.node_len), r.voff, r.vlen);
        } while (next_record(p));
    }
    p.ws();
    if (p.i != len) throw JsonError();
    return CRDT_HOST_OK;
}

// ---- parallel decode of a large document (CRDT_HOST_THREADS, default min(16, cores)).
// Phase 1, one thread per byte range: the range's first record starts at the first `},"`
// after its nominal start (speculative: the previous range verifies that its own parse ends
// exactly there, else the rest is decoded sequentially); records are parsed into local
// columns and their keys looked up (read-only) in the key table.  Phase 2, in order: node and
// key ids are assigned and repeated keys folded exactly as the sequential decoder does.
struct Chunk {
    uint64_t beg = 0, lim = 0, stop = 0;   // parse from beg; records starting before lim; stop = where it ended
    bool closed = false;                   // ended at the document's closing '}'
    int status = CRDT_HOST_OK;
    std::string karena;                    // decoded key bytes
    std::vector<uint64_t> koff, khash;
    std::vector<uint32_t> klen, kid, nid, vlen;
    std::vector<int64_t> lt;
    std::vector<uint64_t> voff;
    std::vector<std::string> nodes;        // local node ids, first-seen order
};

void parse_chunk(const char* js, uint64_t len, const crdt_keys* keys, Chunk& c) {
    Parser p{js, len, c.beg, std::string()};
    std::string key, node;
    std::unordered_map<std::string, uint32_t> nix;
    RecordText r;
    try {
        do {
            if (p.i >= c.lim) break;
            parse_record(p, js, key, node, r);
            const uint64_t h = hash_bytes(key.data(), key.size());
            uint32_t id;
            if (!keys->find(key.data(), key.size(), h, &id)) id = UINT32_MAX;
            c.koff.push_back(c.karena.size());
            c.karena.append(key);
            c.klen.push_back((uint32_t)key.size());
            c.khash.push_back(h);
            c.kid.push_back(id);
            c.lt.push_back(r.lt);
            auto it = nix.find(node);
            uint32_t ln;
            if (it == nix.end()) {
                ln = (uint32_t)c.nodes.size();
                nix.emplace(node, ln);
                c.nodes.push_back(node);
            } else {
                ln = it->second;
            }
            c.nid.push_back(ln);
            c.voff.push_back(r.voff);
            c.vlen.push_back(r.vlen);
            if (!next_record(p)) { c.closed = true; break; }
        } while (true);
        c.stop = p.i;
    } catch (const Fallback&) {
        c.status = CRDT_HOST_FALLBACK;
    } catch (const JsonError&) {
        c.status = CRDT_HOST_E_JSON;
    } catch (const std::bad_alloc&) {
        c.status = CRDT_HOST_E_NOMEM;
    }
}

int host_threads() {
    if (const char* e = getenv("CRDT_HOST_THREADS")) {
        const int v = atoi(e);
        if (v >= 1) return v < 64 ? v : 64;
    }
    const unsigned hc = std::thread::hardware_concurrency();
    return hc == 0 ? 1 : (hc < 16 ? (int)hc : 16);
}

// fn(chunk, begin, end) over [0, n) split into at most host_threads() chunks of >= min_per items
// (the caller's thread runs chunk 0); returns the number of chunks.
template <typename F>
int parallel_chunks(uint64_t n, uint64_t min_per, F fn) {
    int nt = host_threads();
    if (const char* env = getenv("CRDT_HOST_MIN_CHUNK")) min_per = strtoull(env, nullptr, 10);   // tests
    if (min_per == 0) min_per = 1;
    if ((uint64_t)nt > n / min_per) nt = (int)std::max<uint64_t>(1, n / min_per);
    const uint64_t per = (n + nt - 1) / std::max(nt, 1);
    std::vector<std::thread> pool;
    for (int k = 1; k < nt; ++k) {
        const uint64_t b = std::min<uint64_t>(n, k * per), e = std::min<uint64_t>(n, b + per);
        pool.emplace_back(fn, k, b, e);
    }
    fn(0, 0, std::min<uint64_t>(n, per));
    for (auto& t : pool) t.join();
    return nt;
}

uint64_t parallel_min_bytes() {                       // CRDT_HOST_PAR_MIN: tests split small documents
    if (const char* e = getenv("CRDT_HOST_PAR_MIN")) return strtoull(e, nullptr, 10);
    return 4ull << 20;
}

// Fault in the reserved (not yet written) capacity of the ordered pass's columns from all threads
// at once, so the sequential pass does not take one page fault per 4 KB it appends.
// MADV_POPULATE_WRITE (Linux 5.14); where the kernel lacks it the pages fault as before.
// CRDT_HOST_PREFAULT=0 turns it off (A/B measurement).
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif
struct Span { char* p; uint64_t n; };

template <typename T>
Span spare(std::vector<T>& v) {
    return Span{reinterpret_cast<char*>(v.data() + v.size()), (uint64_t)(v.capacity() - v.size()) * sizeof(T)};
}

void prefault(const std::vector<Span>& spans) {
    if (const char* e = getenv("CRDT_HOST_PREFAULT")) if (e[0] == '0') return;
    const uint64_t pg = (uint64_t)sysconf(_SC_PAGESIZE);
    std::vector<Span> pages;                          // page-aligned pieces of <= 2 MB
    for (const Span& s : spans) {
        uint64_t a = ((uint64_t)s.p + pg - 1) & ~(pg - 1);
        const uint64_t e = ((uint64_t)s.p + s.n) & ~(pg - 1);
        for (; a < e; a += 2ull << 20) pages.push_back(Span{(char*)a, std::min<uint64_t>(2ull << 20, e - a)});
    }
    if (pages.empty()) return;
    parallel_chunks(pages.size(), 1, [&](int, uint64_t b, uint64_t e) {
        for (uint64_t k = b; k < e; ++k) madvise(pages[k].p, pages[k].n, MADV_POPULATE_WRITE);
    });
}

int decode_parallel(const char* js, uint64_t len, crdt_keys* keys, crdt_decoded* d, int nthreads) {
    Parser p0{js, len, 0, std::string()};
    begin_object(p0);
    if (p0.peek() == '}') return decode_sequential(js, len, keys, d);
    const uint64_t first = p0.i;
    // chunk starts: chunk 0 at the first key; chunk k at the first `},"` after k * len / n
    std::vector<uint64_t> starts{first};
    for (int k = 1; k < nthreads; ++k) {
        uint64_t g = std::max<uint64_t>((uint64_t)k * (len / nthreads), starts.back() + 1);
        const char* f = nullptr;
        while (g + 3 < len) {
            f = static_cast<const char*>(memchr(js + g, '}', len - g));
            if (!f) break;
            const uint64_t q = f - js;
            uint64_t r = q + 1;
            while (r < len && (js[r] == ' ' || js[r] == '\t' || js[r] == '\n' || js[r] == '\r')) ++r;
            if (r < len && js[r] == ',') {
                ++r;
                while (r < len && (js[r] == ' ' || js[r] == '\t' || js[r] == '\n' || js[r] == '\r')) ++r;
                if (r < len && js[r] == '"') { g = r; break; }
            }
            g = q + 1;
            f = nullptr;
        }
        if (!f) break;
        starts.push_back(g);
    }
    const int n = (int)starts.size();
    std::vector<Chunk> ch(n);
    for (int k = 0; k < n; ++k) {
        ch[k].beg = starts[k];
        ch[k].lim = k + 1 < n ? starts[k + 1] : UINT64_MAX;
    }
    {
        std::vector<std::thread> pool;
        for (int k = 1; k < n; ++k) pool.emplace_back(parse_chunk, js, len, keys, std::ref(ch[k]));
        parse_chunk(js, len, keys, ch[0]);
        for (auto& t : pool) t.join();
    }
    // phase 2: chunks in order while each one's parse was valid and ended where the next began
    Builder bld(keys, d);
    // the key table grows by at most the phase-1 misses (records whose key it did not hold):
    // reserve and prefault that much only, so a re-sync of known keys leaves it as it was; the
    // per-call columns are reserved (and prefaulted) for every record and freed after the call
    uint64_t total = 0, miss = 0, mbytes = 0;
    for (const auto& c : ch) {
        total += c.kid.size();
        for (size_t m = 0; m < c.kid.size(); ++m)
            if (c.kid[m] == UINT32_MAX) { ++miss; mbytes += c.klen[m]; }
    }
    keys->reserve(miss, mbytes);
    d->key.reserve(total); d->lt.reserve(total); d->node.reserve(total); d->voff.reserve(total); d->vlen.reserve(total);
    bld.first_new.reserve(miss);
    std::vector<Span> spans{spare(d->key), spare(d->lt), spare(d->node), spare(d->voff), spare(d->vlen),
                            spare(bld.first_new)};
    if (miss) {                                           // (the table's spare beyond the misses stays virtual)
        spans.push_back(spare(keys->arena));
        spans.push_back(spare(keys->off));
        spans.push_back(spare(keys->hash));
    }
    prefault(spans);
    uint64_t resume = 0;                                  // != 0: decode sequentially from here
    bool closed = false;
    std::vector<uint32_t> nmap;
    for (int k = 0; k < n; ++k) {
        const Chunk& c = ch[k];
        if (c.status == CRDT_HOST_E_NOMEM) throw std::bad_alloc();
        if (c.status == CRDT_HOST_FALLBACK) throw Fallback();   // valid start: this record is the first
        if (c.status == CRDT_HOST_E_JSON) throw JsonError();    // failing one in document order
        nmap.resize(c.nodes.size());
        for (size_t m = 0; m < c.nodes.size(); ++m) nmap[m] = bld.node_id(c.nodes[m].data(), c.nodes[m].size());
        const size_t nr = c.kid.size();
        for (size_t m = 0; m < nr; ++m) {
            if (m + 16 < nr) {                        // the table / first-record probes are cache misses
                if (c.kid[m + 16] == UINT32_MAX) keys->prefetch(c.khash[m + 16]);
                else bld.seen.prefetch(c.kid[m + 16]);
            }
            bld.add(c.karena.data() + c.koff[m], c.klen[m], c.khash[m], c.kid[m], c.lt[m], nmap[c.nid[m]], c.voff[m],
                    c.vlen[m]);
        }
        if (c.closed) { closed = true; break; }
        if (k + 1 < n && c.stop != starts[k + 1]) { resume = c.stop; break; }   // speculation failed
        if (k + 1 == n) resume = c.stop;                  // (cannot happen: the last chunk has no limit)
    }
    if (!closed) {
        // the rest, sequentially, from a verified record start
        Parser p{js, len, resume, std::string()};
        std::string key, node;
        RecordText r;
        do {
            parse_record(p, js, key, node, r);
            bld.add(key.data(), key.size(), hash_bytes(key.data(), key.size()), UINT32_MAX, r.lt,
                    bld.node_id(r.node, r.node_len), r.voff, r.vlen);
        } while (next_record(p));
        closed = true;
        p0.i = p.i;
    } else {
        // find where the closing '}' left the parse: the last used chunk's stop
        for (int k = 0; k < n; ++k)
            if (ch[k].closed) { p0.i = ch[k].stop; break; }
    }
    p0.ws();
    if (p0.i != len) throw JsonError();
    return CRDT_HOST_OK;
}

int decode(const char* js, uint64_t len, crdt_keys* keys, crdt_decoded* d) {
    const uint64_t n0 = keys->size();
    try {
        const int nt = len >= parallel_min_bytes() ? host_threads() : 1;
        return nt > 1 ? decode_parallel(js, len, keys, d, nt) : decode_sequential(js, len, keys, d);
    } catch (const Fallback&) {
        crdt_keys_truncate(keys, n0);
        return CRDT_HOST_FALLBACK;
    } catch (const JsonError&) {
        crdt_keys_truncate(keys, n0);
        return CRDT_HOST_E_JSON;
    } catch (const std::bad_alloc&) {
        crdt_keys_truncate(keys, n0);
        return CRDT_HOST_E_NOMEM;
    }
}

}  // namespace


namespace {

// ------------------------------------------------------------------ export helpers
// Hlc.toString's fixed 30-byte head "YYYY-MM-DDTHH:MM:SS.mmmZ-XXXX-" of Hlc.fromLogicalTime(lt)
// (hlc.dart:37, 101-104); false outside years 0000..9999 (Dart's +/-YYYYYY forms).
bool hlc_head(int64_t lt, char* q) {
    static const char hx[] = "0123456789ABCDEF";
    const int64_t ms = lt >> kShift;
    const int64_t counter = lt & 0xFFFF;
    if (ms > kMaxMs || ms < -kMaxMs) return false;
    const int64_t days = floordiv(ms, 86400000);
    int64_t rem = ms - days * 86400000;
    int64_t y, mo, d;
    civil_from_days(days, &y, &mo, &d);
    if (y < 0 || y > 9999) return false;
    const int64_t h = rem / 3600000;
    rem -= h * 3600000;
    const int64_t mi = rem / 60000;
    rem -= mi * 60000;
    const int64_t s = rem / 1000, milli = rem - s * 1000;
    q[0] = '0' + y / 1000; q[1] = '0' + y / 100 % 10; q[2] = '0' + y / 10 % 10; q[3] = '0' + y % 10;
    q[4] = '-'; q[5] = '0' + mo / 10; q[6] = '0' + mo % 10; q[7] = '-'; q[8] = '0' + d / 10; q[9] = '0' + d % 10;
    q[10] = 'T'; q[11] = '0' + h / 10; q[12] = '0' + h % 10; q[13] = ':'; q[14] = '0' + mi / 10;
    q[15] = '0' + mi % 10; q[16] = ':'; q[17] = '0' + s / 10; q[18] = '0' + s % 10; q[19] = '.';
    q[20] = '0' + milli / 100; q[21] = '0' + milli / 10 % 10; q[22] = '0' + milli % 10; q[23] = 'Z';
    q[24] = '-';
    q[25] = hx[(counter >> 12) & 15]; q[26] = hx[(counter >> 8) & 15]; q[27] = hx[(counter >> 4) & 15];
    q[28] = hx[counter & 15];
    q[29] = '-';
    return true;
}

// String body escaped as jsonEncode / json.dumps(ensure_ascii=False) write it: '"', '\\' and
// the C0 controls (\b \t \n \f \r short, the rest \u00xx); every other byte verbatim.
void json_escape(std::string& o, const char* p, uint64_t n) {
    static const char hx[] = "0123456789abcdef";
    uint64_t run = 0;
    for (uint64_t k = 0; k < n; ++k) {
        const uint8_t c = (uint8_t)p[k];
        if (c >= 0x20 && c != '"' && c != '\\') continue;
        o.append(p + run, k - run);
        run = k + 1;
        switch (c) {
            case '"': o += "\\\""; break;
            case '\\': o += "\\\\"; break;
            case '\b': o += "\\b"; break;
            case '\t': o += "\\t"; break;
            case '\n': o += "\\n"; break;
            case '\f': o += "\\f"; break;
            case '\r': o += "\\r"; break;
            default: {
                const char u[6] = {'\\', 'u', '0', '0', hx[c >> 4], hx[c & 15]};
                o.append(u, 6);
            }
        }
    }
    o.append(p + run, n - run);
}

// Is text == json.dumps(json.loads(text), separators=(',', ':'), ensure_ascii=False)?  Then a
// raw input span can be exported verbatim.  Conservative: any float, "-0", whitespace, an
// escape dumps would not write, a repeated object key, a surrogate, invalid UTF-8 or a very
// deep / very long number answers no (the caller then re-encodes that value).
struct Canon {
    const char* s;
    uint64_t n, i = 0;

    bool utf8_char() {                        // s[i] >= 0x80: one well-formed non-surrogate scalar
        const uint8_t c = (uint8_t)s[i];
        int len;
        uint32_t cp;
        if (c >= 0xC2 && c <= 0xDF) { len = 2; cp = c & 0x1F; }
        else if (c >= 0xE0 && c <= 0xEF) { len = 3; cp = c & 0x0F; }
        else if (c >= 0xF0 && c <= 0xF4) { len = 4; cp = c & 0x07; }
        else return false;
        if (i + len > n) return false;
        for (int k = 1; k < len; ++k) {
            const uint8_t t = (uint8_t)s[i + k];
            if ((t & 0xC0) != 0x80) return false;
            cp = (cp << 6) | (t & 0x3F);
        }
        if ((len == 3 && (cp < 0x800 || (cp >= 0xD800 && cp < 0xE000))) || (len == 4 && (cp < 0x10000 || cp > 0x10FFFF)))
            return false;
        i += len;
        return true;
    }

    bool string() {
        if (i >= n || s[i] != '"') return false;
        ++i;
        while (i < n) {
            const uint8_t c = (uint8_t)s[i];
            if (c == '"') { ++i; return true; }
            if (c < 0x20) return false;
            if (c >= 0x80) {
                if (!utf8_char()) return false;
                continue;
            }
            if (c == '\\') {
                if (i + 1 >= n) return false;
                const char e = s[i + 1];
                if (e == '"' || e == '\\' || e == 'b' || e == 'f' || e == 'n' || e == 'r' || e == 't') {
                    i += 2;
                    continue;
                }
                // dumps writes \u00xx (lowercase) only for controls without a short form
                if (e != 'u' || i + 6 > n || s[i + 2] != '0' || s[i + 3] != '0') return false;
                const char a = s[i + 4], b = s[i + 5];
                if (a != '0' && a != '1') return false;
                if (!((b >= '0' && b <= '9') || (b >= 'a' && b <= 'f'))) return false;
                const int v = (a - '0') * 16 + hexval(b);
                if (v == 8 || v == 9 || v == 10 || v == 12 || v == 13) return false;
                i += 6;
                continue;
            }
            ++i;
        }
        return false;
    }

    bool number() {
        const uint64_t b = i;
        if (s[i] == '-') ++i;
        if (i >= n) return false;
        if (s[i] == '0') {
            ++i;
            if (i - b == 2) return false;             // "-0" loads as int 0
        } else if (s[i] >= '1' && s[i] <= '9') {
            while (i < n && s[i] >= '0' && s[i] <= '9') ++i;
        } else {
            return false;
        }
        if (i < n && (s[i] == '.' || s[i] == 'e' || s[i] == 'E')) return false;   // floats re-print
        return i - b <= 4000;                         // Python's int string-length limit
    }

    bool lit(const char* w, uint64_t l) {
        if (i + l > n || memcmp(s + i, w, l) != 0) return false;
        i += l;
        return true;
    }

    bool value(int depth) {
        if (depth > 400 || i >= n) return false;
        const char c = s[i];
        if (c == '{') {
            ++i;
            if (i < n && s[i] == '}') { ++i; return true; }
            std::vector<std::string_view> ks;
            std::unordered_set<std::string_view> big;
            while (true) {
                const uint64_t kb = i;
                if (!string()) return false;
                const std::string_view k(s + kb, i - kb);     // canonical: equal bytes <=> equal keys
                if (big.empty() && ks.size() < 16) {
                    for (const auto& x : ks)
                        if (x == k) return false;
                    ks.push_back(k);
                } else {
                    if (big.empty()) big.insert(ks.begin(), ks.end());
                    if (!big.insert(k).second) return false;
                }
                if (i >= n || s[i] != ':') return false;
                ++i;
                if (!value(depth + 1)) return false;
                if (i < n && s[i] == ',') { ++i; continue; }
                if (i < n && s[i] == '}') { ++i; return true; }
                return false;
            }
        }
        if (c == '[') {
            ++i;
            if (i < n && s[i] == ']') { ++i; return true; }
            while (true) {
                if (!value(depth + 1)) return false;
                if (i < n && s[i] == ',') { ++i; continue; }
                if (i < n && s[i] == ']') { ++i; return true; }
                return false;
            }
        }
        if (c == '"') return string();
        if (c == 't') return lit("true", 4);
        if (c == 'f') return lit("false", 5);
        if (c == 'n') return lit("null", 4);
        if (c == '-' || (c >= '0' && c <= '9')) return number();
        return false;
    }
};

}  // namespace

struct crdt_text {
    std::string s;
};

extern "C" {

int crdt_host_abi_version(void) { return CRDT_HOST_ABI_VERSION; }

crdt_keys* crdt_keys_create(void) { return new (std::nothrow) crdt_keys(); }
void crdt_keys_destroy(crdt_keys* k) { delete k; }
uint64_t crdt_keys_size(const crdt_keys* k) { return k ? k->size() : 0; }

int crdt_keys_find(const crdt_keys* k, const char* p, uint64_t n, uint32_t* id) {
    if (!k || (!p && n) || !id) return CRDT_HOST_E_INVALID;
    return k->find(p, n, hash_bytes(p, n), id) ? 0 : 1;
}

int crdt_keys_intern(crdt_keys* k, const char* p, uint64_t n, uint32_t* id, int* is_new) {
    if (!k || (!p && n) || !id) return CRDT_HOST_E_INVALID;
    const uint64_t h = hash_bytes(p, n);
    try {
        const bool found = k->find(p, n, h, id);
        if (!found) {
            if (k->size() >= 0xFFFFFFF0ull) return CRDT_HOST_E_NOMEM;
            *id = k->add(p, n, h);
        }
        if (is_new) *is_new = found ? 0 : 1;
    } catch (const std::bad_alloc&) {
        return CRDT_HOST_E_NOMEM;
    }
    return CRDT_HOST_OK;
}

uint64_t crdt_keys_bytes(const crdt_keys* k, uint64_t first, uint64_t count) {
    if (!k || first + count > k->size()) return 0;
    return k->off[first + count] - k->off[first];
}

int crdt_keys_export(const crdt_keys* k, uint64_t first, uint64_t count, char* buf, uint64_t cap,
                     uint64_t* offsets) {
    if (!k || !offsets || first + count > k->size()) return CRDT_HOST_E_INVALID;
    const uint64_t b = k->off[first], e = k->off[first + count];
    if (e - b > cap || (!buf && e > b)) return CRDT_HOST_E_INVALID;
    if (e > b) memcpy(buf, k->arena.data() + b, e - b);
    for (uint64_t i = 0; i <= count; ++i) offsets[i] = k->off[first + i] - b;
    return CRDT_HOST_OK;
}

int crdt_keys_truncate(crdt_keys* k, uint64_t n) {
    if (!k) return CRDT_HOST_E_INVALID;
    if (n >= k->size()) return CRDT_HOST_OK;
    k->arena.resize(k->off[n]);
    k->off.resize(n + 1);
    k->hash.resize(n);
    k->rebuild(n > 8 ? n : 8);
    return CRDT_HOST_OK;
}

int crdt_keys_clear(crdt_keys* k) { return crdt_keys_truncate(k, 0); }

int crdt_json_decode(const char* json, uint64_t len, crdt_keys* keys, crdt_decoded** out) {
    if (!keys || !out || (!json && len)) return CRDT_HOST_E_INVALID;
    *out = nullptr;
    crdt_decoded* d = new (std::nothrow) crdt_decoded();
    if (!d) return CRDT_HOST_E_NOMEM;
    const int st = decode(json, len, keys, d);
    if (st != CRDT_HOST_OK) {
        delete d;
        return st;
    }
    *out = d;
    return CRDT_HOST_OK;
}

void crdt_decoded_free(crdt_decoded* d) { delete d; }
uint64_t crdt_decoded_count(const crdt_decoded* d) { return d ? d->key.size() : 0; }
uint32_t crdt_decoded_node_count(const crdt_decoded* d) { return d ? (uint32_t)d->nodes.size() : 0; }

int crdt_decoded_columns(const crdt_decoded* d, uint32_t* key_id, int64_t* lt, uint32_t* node, uint64_t* val_off,
                         uint32_t* val_len) {
    if (!d) return CRDT_HOST_E_INVALID;
    const size_t n = d->key.size();
    if (key_id) memcpy(key_id, d->key.data(), n * 4);
    if (lt) memcpy(lt, d->lt.data(), n * 8);
    if (node) memcpy(node, d->node.data(), n * 4);
    if (val_off) memcpy(val_off, d->voff.data(), n * 8);
    if (val_len) memcpy(val_len, d->vlen.data(), n * 4);
    return CRDT_HOST_OK;
}

uint64_t crdt_decoded_node_bytes(const crdt_decoded* d) {
    uint64_t b = 0;
    if (d)
        for (const auto& s : d->nodes) b += s.size();
    return b;
}

int crdt_decoded_nodes(const crdt_decoded* d, char* buf, uint64_t cap, uint64_t* offsets) {
    if (!d || !offsets) return CRDT_HOST_E_INVALID;
    uint64_t o = 0;
    offsets[0] = 0;
    for (size_t i = 0; i < d->nodes.size(); ++i) {
        const std::string& s = d->nodes[i];
        if (o + s.size() > cap) return CRDT_HOST_E_INVALID;
        if (!s.empty()) memcpy(buf + o, s.data(), s.size());
        o += s.size();
        offsets[i + 1] = o;
    }
    return CRDT_HOST_OK;
}

int crdt_hlc_format(const int64_t* lt, const uint32_t* node, uint64_t n, const char* node_buf,
                    const uint64_t* node_off, char* out, uint64_t cap, uint64_t* out_off) {
    if ((!lt || !node || !node_off || !out_off) && n) return CRDT_HOST_E_INVALID;
    uint64_t o = 0;
    out_off[0] = 0;
    for (uint64_t i = 0; i < n; ++i) {
        const uint64_t nb = node_off[node[i]], ne = node_off[node[i] + 1];
        if (o + 30 + (ne - nb) > cap) return CRDT_HOST_E_INVALID;
        if (!hlc_head(lt[i], out + o)) return CRDT_HOST_FALLBACK;
        if (ne > nb) memcpy(out + o + 30, node_buf + nb, ne - nb);
        o += 30 + (ne - nb);
        out_off[i + 1] = o;
    }
    return CRDT_HOST_OK;
}

int crdt_json_canonical(const char* buf, const uint64_t* off, const uint32_t* len, uint64_t n, uint8_t* ok) {
    if ((!buf || !off || !len || !ok) && n) return CRDT_HOST_E_INVALID;
    std::vector<int> st(64, CRDT_HOST_OK);
    parallel_chunks(n, 16384, [&](int ch, uint64_t b, uint64_t e) {
        try {
            for (uint64_t k = b; k < e; ++k) {
                Canon c{buf + off[k], len[k]};
                ok[k] = len[k] > 0 && c.value(0) && c.i == c.n;
            }
        } catch (const std::bad_alloc&) {
            st[ch] = CRDT_HOST_E_NOMEM;
        }
    });
    for (int v : st)
        if (v != CRDT_HOST_OK) return v;
    return CRDT_HOST_OK;
}

int crdt_json_split(const char* json, uint64_t len, uint64_t count, uint64_t* off, uint32_t* elen) {
    if ((!json && len) || ((!off || !elen) && count)) return CRDT_HOST_E_INVALID;
    Parser p{json, len};
    try {
        p.expect('[');
        uint64_t k = 0;
        if (p.peek() == ']') {
            ++p.i;
        } else {
            while (true) {
                const uint64_t b = p.i;
                p.skip_value(0);
                if (k >= count || p.i - b > 0xFFFFFFFFull) return CRDT_HOST_FALLBACK;
                off[k] = b;
                elen[k] = (uint32_t)(p.i - b);
                ++k;
                if (p.peek() == ',') { ++p.i; continue; }
                p.expect(']');
                break;
            }
        }
        if (k != count || p.i != len) return CRDT_HOST_FALLBACK;
    } catch (const JsonError&) {
        return CRDT_HOST_E_JSON;
    } catch (const Fallback&) {
        return CRDT_HOST_FALLBACK;
    }
    return CRDT_HOST_OK;
}

int crdt_json_encode(const crdt_keys* keys, const uint32_t* key_id, const int64_t* lt, const uint32_t* node,
                     const char* const* hlc_txt, const uint32_t* hlc_len, const char* const* val_txt,
                     const uint32_t* val_len, uint64_t n, const char* node_buf, const uint64_t* node_off,
                     uint32_t n_nodes, crdt_text** out) {
    if (!keys || !out || ((!key_id || !lt || !node || !val_len || !node_off) && n)) return CRDT_HOST_E_INVALID;
    *out = nullptr;
    crdt_text* t = new (std::nothrow) crdt_text();
    if (!t) return CRDT_HOST_E_NOMEM;
    // records [b, e) into part `ch` (rows 1.. of a part start with ','), parts concatenated
    std::vector<std::string> parts(64);
    std::vector<int> st(64, CRDT_HOST_OK);
    const int np = parallel_chunks(n, 32768, [&](int ch, uint64_t b, uint64_t e) {
        try {
            std::string& o = parts[ch];
            uint64_t want = 0;
            for (uint64_t i = b; i < e; ++i) want += 64 + val_len[i];
            o.reserve(want + want / 8);
            char head[30];
            for (uint64_t i = b; i < e; ++i) {
                const uint32_t id = key_id[i];
                if (id >= keys->size() || node[i] >= n_nodes || (val_len[i] && (!val_txt || !val_txt[i]))) {
                    st[ch] = CRDT_HOST_E_INVALID;
                    return;
                }
                if (i) o += ',';
                o += '"';
                json_escape(o, keys->arena.data() + keys->off[id], keys->off[id + 1] - keys->off[id]);
                o += "\":{\"hlc\":\"";
                if (hlc_txt && hlc_txt[i]) {                // an Hlc not in columnar form (caller-made)
                    json_escape(o, hlc_txt[i], hlc_len[i]);
                } else {
                    if (!hlc_head(lt[i], head)) {
                        st[ch] = CRDT_HOST_FALLBACK;
                        return;
                    }
                    o.append(head, 30);
                    json_escape(o, node_buf + node_off[node[i]], node_off[node[i] + 1] - node_off[node[i]]);
                }
                o += "\",\"value\":";
                if (val_len[i]) o.append(val_txt[i], val_len[i]);
                else o += "null";
                o += '}';
            }
        } catch (const std::bad_alloc&) {
            st[ch] = CRDT_HOST_E_NOMEM;
        }
    });
    for (int k = 0; k < np; ++k)
        if (st[k] != CRDT_HOST_OK) {
            delete t;
            return st[k];
        }
    try {
        uint64_t total = 2;
        for (int k = 0; k < np; ++k) total += parts[k].size();
        t->s.reserve(total);
        t->s += '{';
        for (int k = 0; k < np; ++k) t->s += parts[k];
        t->s += '}';
    } catch (const std::bad_alloc&) {
        delete t;
        return CRDT_HOST_E_NOMEM;
    }
    *out = t;
    return CRDT_HOST_OK;
}

const char* crdt_text_data(const crdt_text* t) { return t ? t->s.data() : nullptr; }
uint64_t crdt_text_size(const crdt_text* t) { return t ? t->s.size() : 0; }
void crdt_text_free(crdt_text* t) { delete t; }

}  // extern "C"
