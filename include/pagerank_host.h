/*
 * libpagerank_host -- native host front-end and writers of the drop-in (C ABI, CPU only).
 *
 * Replaces the reference's input/output stages around the hot path:
 *   input   Sparky.java:61-123  sequenceFile(url, json) -> link extraction -> (url, href|null)
 *           or a plain edge list "src dst" / "src" (the north-star CLI input);
 *   interning (first appearance, src before dst) to the dense int32 IDs libpagerank_hip takes;
 *   output  Sparky.java:237 saveAsTextFile -> "(url,rank)" part files, and the north-star
 *           "<url> has rank: <r>." lines, both with Java Double.toString.
 * Every function returns 0 or a negative code; prh_last_error() holds the message.
 */
#ifndef PAGERANK_HOST_H
#define PAGERANK_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PRH_FORMAT_EDGES 0  /* "src dst" per line; "src" alone = record without links     */
#define PRH_FORMAT_CCJSON 1 /* "url<TAB>json" per line: Common Crawl metadata records
                               (the Text/Text pairs of Sparky.java:61), links extracted as in
                               Sparky.java:87-118 with Gson's JsonElement.toString() quirks  */

typedef struct prh_edges prh_edges;

const char *prh_last_error(void);
int prh_read(const char *path, int32_t format, prh_edges **out);
/* Threads of the edge-list reader (PRH_FORMAT_EDGES): 0 = automatic (one for inputs under 16 MiB,
   else the host's granted cores, at most 64).  The IDs are the same for any count: first
   appearance in file order, src before dst. */
void prh_set_read_threads(int32_t n);
/* the same from a memory buffer (tests, embedding) */
int prh_parse(const char *data, int64_t len, int32_t format, prh_edges **out);
int64_t prh_n_edges(const prh_edges *e);
int32_t prh_n_vertices(const prh_edges *e);
const int32_t *prh_src(const prh_edges *e); /* n_edges interned IDs                        */
const int32_t *prh_dst(const prh_edges *e); /* n_edges, -1 = record without links          */
const char *prh_name(const prh_edges *e, int32_t id, int64_t *len); /* not NUL-terminated */
/* Java Double.toString into buf (>= 40 bytes); returns the length. */
int32_t prh_java_double(double x, char *buf);
/* dir/PageRank<iter>/part-00000 with "(url,rank)" lines + empty _SUCCESS. */
int prh_write_part(const prh_edges *e, const char *dir, int32_t iter, const double *ranks);
/* "<url> has rank: <r>." for every URL, to path (NULL = stdout). */
int prh_write_has_rank(const prh_edges *e, const char *path, const double *ranks);
/* Resume: ranks[id] from the "(url,rank)" lines of every dir/part-* file (a PageRank<i>
   directory written by prh_write_part or by Sparky.java:237's saveAsTextFile).  Every URL of
   the edge list must appear exactly once, and only those. */
int prh_read_ranks(const prh_edges *e, const char *dir, double *ranks);
void prh_free(prh_edges *e);

#ifdef __cplusplus
}
#endif

#endif /* PAGERANK_HOST_H */
