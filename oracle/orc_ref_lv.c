/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see orc_lv.h).
 *
 * Adapter from the oracle's lv_* interface onto the REFERENCE's own libVig,
 * compiled unmodified from /root/reference/libvig/verified/*.c by
 * oracle/Makefile (target `ref`) into oracle/_ref/liborc_ref.so. Nothing here
 * re-implements libVig: every call forwards to the reference function of the
 * same name. The reference has no destructors, so lv_*_free leak (tests keep
 * capacities small).
 */
#include <stdlib.h>

#include "orc_lv.h"

#include "libvig/verified/cht.h"
#include "libvig/verified/double-chain.h"
#include "libvig/verified/expirator.h"
#include "libvig/verified/map.h"
#include "libvig/verified/vector.h"

const char *lv_impl_name(void) { return "reference"; }

int lv_map_allocate(lv_eq_fn *eq, lv_hash_fn *hash, unsigned capacity,
                    struct lv_map **out) {
  struct Map *m = NULL;
  if (!map_allocate((map_keys_equality *)eq, (map_key_hash *)hash, capacity, &m))
    return 0;
  *out = (struct lv_map *)m;
  return 1;
}
int lv_map_get(struct lv_map *m, void *key, int *value_out) {
  return map_get((struct Map *)m, key, value_out);
}
void lv_map_put(struct lv_map *m, void *key, int value) {
  map_put((struct Map *)m, key, value);
}
void lv_map_erase(struct lv_map *m, void *key, void **trash) {
  map_erase((struct Map *)m, key, trash);
}
unsigned lv_map_size(struct lv_map *m) { return map_size((struct Map *)m); }
void lv_map_free(struct lv_map *m) { (void)m; }

int lv_dchain_allocate(int index_range, struct lv_dchain **out) {
  struct DoubleChain *c = NULL;
  if (!dchain_allocate(index_range, &c)) return 0;
  *out = (struct lv_dchain *)c;
  return 1;
}
int lv_dchain_allocate_new_index(struct lv_dchain *c, int *index_out,
                                 lv_time_t t) {
  return dchain_allocate_new_index((struct DoubleChain *)c, index_out, t);
}
int lv_dchain_rejuvenate_index(struct lv_dchain *c, int index, lv_time_t t) {
  return dchain_rejuvenate_index((struct DoubleChain *)c, index, t);
}
int lv_dchain_expire_one_index(struct lv_dchain *c, int *index_out,
                               lv_time_t t) {
  return dchain_expire_one_index((struct DoubleChain *)c, index_out, t);
}
int lv_dchain_is_index_allocated(struct lv_dchain *c, int index) {
  return dchain_is_index_allocated((struct DoubleChain *)c, index);
}
int lv_dchain_free_index(struct lv_dchain *c, int index) {
  return dchain_free_index((struct DoubleChain *)c, index);
}
void lv_dchain_free(struct lv_dchain *c) { (void)c; }

/* Observability only: walks the reference's cells through the struct layout
 * it declares at libvig/verified/double-chain.c:16-19 and
 * double-chain-impl.h:6-9 ({int prev, next}; heads at cells 0 and 1). */
struct ref_dchain_view {
  struct {
    int prev, next;
  } *cells;
  lv_time_t *timestamps;
};
int lv_dchain_dump(struct lv_dchain *c, int index_range, int *alloc_order,
                   int *n_alloc, int *free_order, int *n_free, lv_time_t *ts) {
  struct ref_dchain_view *v = (struct ref_dchain_view *)c;
  int k = 0;
  for (int x = v->cells[0].next; x != 0 && k < index_range; x = v->cells[x].next)
    alloc_order[k++] = x - 2;
  *n_alloc = k;
  k = 0;
  for (int x = v->cells[1].next; x != 1 && k < index_range; x = v->cells[x].next)
    free_order[k++] = x - 2;
  *n_free = k;
  for (int i = 0; i < index_range; i++) ts[i] = v->timestamps[i];
  return 1;
}

int lv_vector_allocate(int elem_size, unsigned capacity, lv_init_fn *init,
                       struct lv_vector **out) {
  struct Vector *v = NULL;
  if (!vector_allocate(elem_size, capacity, (vector_init_elem *)init, &v))
    return 0;
  *out = (struct lv_vector *)v;
  return 1;
}
void lv_vector_borrow(struct lv_vector *v, int index, void **val_out) {
  vector_borrow((struct Vector *)v, index, val_out);
}
void lv_vector_return(struct lv_vector *v, int index, void *val) {
  vector_return((struct Vector *)v, index, val);
}
void lv_vector_free(struct lv_vector *v) { (void)v; }

int lv_expire_items_single_map(struct lv_dchain *c, struct lv_vector *v,
                               struct lv_map *m, lv_time_t t) {
  return expire_items_single_map((struct DoubleChain *)c, (struct Vector *)v,
                                 (struct Map *)m, t);
}

int lv_cht_fill_cht(struct lv_vector *cht, uint32_t height,
                    uint32_t backend_capacity) {
  return cht_fill_cht((struct Vector *)cht, height, backend_capacity);
}
int lv_cht_find_preferred_available_backend(uint64_t hash,
                                            struct lv_vector *cht,
                                            struct lv_dchain *active,
                                            uint32_t height,
                                            uint32_t backend_capacity,
                                            int *chosen) {
  return cht_find_preferred_available_backend(
      hash, (struct Vector *)cht, (struct DoubleChain *)active, height,
      backend_capacity, chosen);
}
