/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into, loaded by, or called
 * from the product path (vigor_amd/, include/). Only tests/, bench.py's
 * cpu_baseline leg and __graft_entry__.smoke() may use it, as the checker.
 *
 * The libVig data-structure interface the oracle's NF glue is written against.
 * Two implementations exist:
 *   oracle/orc_libvig.c   clean-room C restatement (liborc.so)
 *   oracle/orc_ref_lv.c   thin adapter onto the reference's own libVig sources,
 *                         compiled from the reference libvig/verified sources by
 *                         oracle/Makefile into oracle/_ref/liborc_ref.so
 * Same glue + either implementation must produce identical traces; that is how
 * the restatement is pinned to the reference (tests/test_oracle_ref.py).
 *
 * Semantics follow (reference paths relative to /root/reference):
 *   map      libvig/verified/map.c:149-206,238-273, map-impl-pow2.c:629-732,
 *            790-972, 1110-1217 (CAPACITY_POW2 build, Makefile.dpdk:38)
 *   dchain   libvig/verified/double-chain.c:113-913, double-chain-impl.c
 *   vector   libvig/verified/vector.c:147-311
 *   expirator libvig/verified/expirator.c:110-218
 *   cht      libvig/verified/cht.c:546-1062
 */
#ifndef ORC_LV_H
#define ORC_LV_H
#include <stdbool.h>
#include <stdint.h>

typedef int64_t lv_time_t; /* vigor_time_t, libvig/verified/vigor-time.h:7 */

typedef unsigned lv_hash_fn(void *key);       /* map-util.h:13 */
typedef bool lv_eq_fn(void *a, void *b);      /* map-util.h:14 */
typedef void lv_init_fn(void *elem);          /* vector.h */

struct lv_map;
struct lv_dchain;
struct lv_vector;

int lv_map_allocate(lv_eq_fn *eq, lv_hash_fn *hash, unsigned capacity,
                    struct lv_map **out);
int lv_map_get(struct lv_map *m, void *key, int *value_out);
void lv_map_put(struct lv_map *m, void *key, int value);
void lv_map_erase(struct lv_map *m, void *key, void **trash);
unsigned lv_map_size(struct lv_map *m);
void lv_map_free(struct lv_map *m);

int lv_dchain_allocate(int index_range, struct lv_dchain **out);
int lv_dchain_allocate_new_index(struct lv_dchain *c, int *index_out,
                                 lv_time_t t);
int lv_dchain_rejuvenate_index(struct lv_dchain *c, int index, lv_time_t t);
int lv_dchain_expire_one_index(struct lv_dchain *c, int *index_out,
                               lv_time_t t);
int lv_dchain_is_index_allocated(struct lv_dchain *c, int index);
int lv_dchain_free_index(struct lv_dchain *c, int index);
void lv_dchain_free(struct lv_dchain *c);
/* Test observability: alloc list (oldest first), free list (head first) and
 * every timestamp. Arrays are sized index_range. Returns 1. */
int lv_dchain_dump(struct lv_dchain *c, int index_range, int *alloc_order,
                   int *n_alloc, int *free_order, int *n_free, lv_time_t *ts);

int lv_vector_allocate(int elem_size, unsigned capacity, lv_init_fn *init,
                       struct lv_vector **out);
void lv_vector_borrow(struct lv_vector *v, int index, void **val_out);
void lv_vector_return(struct lv_vector *v, int index, void *val);
void lv_vector_free(struct lv_vector *v);

int lv_expire_items_single_map(struct lv_dchain *c, struct lv_vector *v,
                               struct lv_map *m, lv_time_t t);

int lv_cht_fill_cht(struct lv_vector *cht, uint32_t height,
                    uint32_t backend_capacity);
int lv_cht_find_preferred_available_backend(uint64_t hash,
                                            struct lv_vector *cht,
                                            struct lv_dchain *active,
                                            uint32_t height,
                                            uint32_t backend_capacity,
                                            int *chosen);

/* Implementation tag, so a test can tell which build it loaded. */
const char *lv_impl_name(void);

#endif
