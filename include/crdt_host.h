/* crdt_host.h — C-ABI of the native host ingest and export for the MapCrdt merge path.
 *
 * The north star keeps JSON decoding and string interning on the host; this
 * library is that host half, in C++ (crdt_amd/csrc/crdt_host.cpp, built with g++
 * into crdt_amd/libcrdt_host.so, no GPU code).  It replaces, for the common wire
 * format, the per-record work of
 *   Crdt.mergeJson -> CrdtJson.decode -> Record.fromJson -> Hlc.parse
 *   (crdt.dart:100-109, crdt_json.dart:19-37, record.dart:21-26, hlc.dart:39-46)
 * and produces the integer columns crdt_merge (crdt_merge.h) consumes; on the way out it
 * replaces Crdt.toJson -> CrdtJson.encode -> Record.toJson -> Hlc.toString
 * (crdt.dart:127-135, crdt_json.dart:8-17, record.dart:28-31, hlc.dart:101-104) for the rows
 * crdt_modified_since selects (crdt_json_encode).
 *
 * Fast path = what CrdtJson.encode / Hlc.toString emit (crdt_json.dart:8-17,
 * hlc.dart:101-104): {"<key>": {"hlc": "YYYY-MM-DDTHH:MM:SS.mmmZ-XXXX-<node>",
 * "value": <json>}, ...}.  Anything else (other ISO forms, other counter widths, a
 * ':' inside the node id, a non-object record, lone UTF-16 surrogates, ...) returns
 * CRDT_HOST_FALLBACK and the caller decodes with its full restatement, so results
 * never differ from it.
 */
#ifndef CRDT_HOST_H
#define CRDT_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CRDT_HOST_ABI_VERSION 2

enum crdt_host_status {
    CRDT_HOST_OK = 0,
    CRDT_HOST_FALLBACK = 1,       /* valid input outside the fast path: decode it the slow way */
    CRDT_HOST_E_INVALID = -1,     /* bad argument */
    CRDT_HOST_E_JSON = -2,        /* malformed JSON (jsonDecode would throw FormatException) */
    CRDT_HOST_E_NOMEM = -3
};

int crdt_host_abi_version(void);

/* ---- key interning: UTF-8 key string <-> dense uint32 id in first-committed order
 * (the LinkedHashMap insertion order of MapCrdt._map, map_crdt.dart:10). */
typedef struct crdt_keys crdt_keys;
crdt_keys* crdt_keys_create(void);
void crdt_keys_destroy(crdt_keys* k);
uint64_t crdt_keys_size(const crdt_keys* k);
/* 0 found (*id set), 1 absent */
int crdt_keys_find(const crdt_keys* k, const char* utf8, uint64_t len, uint32_t* id);
/* *is_new = 1 when the key got the next id */
int crdt_keys_intern(crdt_keys* k, const char* utf8, uint64_t len, uint32_t* id, int* is_new);
/* bytes of keys [first, first + count) concatenated into buf (capacity cap), offsets[count + 1] */
int crdt_keys_export(const crdt_keys* k, uint64_t first, uint64_t count, char* buf, uint64_t cap,
                     uint64_t* offsets);
uint64_t crdt_keys_bytes(const crdt_keys* k, uint64_t first, uint64_t count);
int crdt_keys_truncate(crdt_keys* k, uint64_t n);     /* forget ids >= n */
int crdt_keys_clear(crdt_keys* k);

/* ---- CrdtJson.decode of one document into columns.
 * Keys are interned into `keys` as they are met (ids of keys new to the table are
 * appended; the caller truncates them if the merge does not store them).  Records
 * are in the document's key order; a key repeated in the document keeps its first
 * position and its last record (jsonDecode into a LinkedHashMap). */
typedef struct crdt_decoded crdt_decoded;
int crdt_json_decode(const char* json, uint64_t len, crdt_keys* keys, crdt_decoded** out);
void crdt_decoded_free(crdt_decoded* d);
uint64_t crdt_decoded_count(const crdt_decoded* d);
uint32_t crdt_decoded_node_count(const crdt_decoded* d);
/* columns, each [count]: key id, Hlc.logicalTime, node index (into the node list),
 * value span in the input (offset, length; length 0 = JSON null or missing = tombstone) */
int crdt_decoded_columns(const crdt_decoded* d, uint32_t* key_id, int64_t* lt, uint32_t* node,
                         uint64_t* val_off, uint32_t* val_len);
/* distinct node ids in first-seen order, UTF-8: bytes into buf (capacity cap), offsets[n + 1] */
uint64_t crdt_decoded_node_bytes(const crdt_decoded* d);
int crdt_decoded_nodes(const crdt_decoded* d, char* buf, uint64_t cap, uint64_t* offsets);

/* ---- Hlc.toString (hlc.dart:101-104) of n clocks whose node ids are given as
 * UTF-8 strings: node_buf/node_off index a node table, node[i] picks the entry.
 * Writes the n strings back to back into out (capacity cap), out_off[n + 1].
 * CRDT_HOST_FALLBACK if some millis is outside years 0000..9999. */
int crdt_hlc_format(const int64_t* lt, const uint32_t* node, uint64_t n, const char* node_buf,
                    const uint64_t* node_off, char* out, uint64_t cap, uint64_t* out_off);

/* ---- export: CrdtJson.encode (crdt_json.dart:8-17) of a recordMap (map_crdt.dart:42-45), one
 * record per row in the given order:
 *   {"<key>":{"hlc":"<Hlc.toString>","value":<value JSON>},...}
 * (Record.toJson, record.dart:28-31; Hlc.toJson = toString, hlc.dart:101-104, 122).  Key i is
 * key_id[i] of `keys`; its hlc is Hlc.fromLogicalTime(lt[i], node table entry node[i]) unless
 * hlc_txt (optional) gives a preformatted text for row i (non-NULL entry); its value is the JSON
 * text val_txt[i][0, val_len[i]) emitted as is (val_len 0 = null, a tombstone).  Keys, node ids
 * and hlc texts are escaped as jsonEncode / json.dumps(ensure_ascii=False) do.  The document is
 * returned in *out (crdt_text_*).  CRDT_HOST_FALLBACK: a millis outside years 0000..9999. */
typedef struct crdt_text crdt_text;
int crdt_json_encode(const crdt_keys* keys, const uint32_t* key_id, const int64_t* lt, const uint32_t* node,
                     const char* const* hlc_txt, const uint32_t* hlc_len, const char* const* val_txt,
                     const uint32_t* val_len, uint64_t n, const char* node_buf, const uint64_t* node_off,
                     uint32_t n_nodes, crdt_text** out);
const char* crdt_text_data(const crdt_text* t);
uint64_t crdt_text_size(const crdt_text* t);
void crdt_text_free(crdt_text* t);

/* ok[k] = 1 when the JSON text buf[off[k], off[k] + len[k]) is exactly what
 * json.dumps(json.loads(text), separators=(',', ':'), ensure_ascii=False) writes back, so a
 * value decoded by crdt_json_decode can be exported verbatim (conservative: floats, "-0",
 * whitespace, escapes dumps would not write, repeated object keys, surrogates answer 0). */
int crdt_json_canonical(const char* buf, const uint64_t* off, const uint32_t* len, uint64_t n, uint8_t* ok);

/* Spans (off, elen) of the `count` elements of one JSON array text (e.g. the values of a batch
 * dumped at once).  CRDT_HOST_FALLBACK when it holds another number of elements or NaN /
 * Infinity / lone surrogates; CRDT_HOST_E_JSON when malformed. */
int crdt_json_split(const char* json, uint64_t len, uint64_t count, uint64_t* off, uint32_t* elen);

#ifdef __cplusplus
}
#endif
#endif /* CRDT_HOST_H */
