/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see orc_lv.h).
 *
 * Clean-room restatement of the libVig data structures the Vigor NFs use on
 * the per-packet path. Written from the behaviour of the reference, cited per
 * function; pinned against the reference's own sources by
 * tests/test_oracle_ref.py (same operation streams through oracle/_ref).
 */
#include <stdlib.h>
#include <stddef.h>
#include <string.h>

#include "orc_lv.h"

const char *lv_impl_name(void) { return "restated"; }

/* ------------------------------------------------------------------ map --
 * Open addressing with linear probing, "chain counters" per slot
 * (libvig/verified/map.c:11-21 SoA layout; map-impl-pow2.c:15-27 `loop` =
 * k & (cap-1)). The map stores key POINTERS (keys live in a vector).
 */
struct lv_map {
  int *busy;       /* busybits */
  void **keyp;     /* keyps */
  unsigned *khash; /* khs */
  int *chain;      /* chns: how many probe chains pass through this slot */
  int *val;        /* vals */
  unsigned cap;
  unsigned size;
  lv_eq_fn *eq;
  lv_hash_fn *hash;
};

int lv_map_allocate(lv_eq_fn *eq, lv_hash_fn *hash, unsigned capacity,
                    struct lv_map **out) {
  /* map.c:56-76: CAPACITY_POW2 requires a non-zero power of two */
  if (capacity == 0 || (capacity & (capacity - 1)) != 0) return 0;
  struct lv_map *m = calloc(1, sizeof *m);
  if (!m) return 0;
  m->busy = calloc(capacity, sizeof(int));
  m->keyp = calloc(capacity, sizeof(void *));
  m->khash = calloc(capacity, sizeof(unsigned));
  m->chain = calloc(capacity, sizeof(int));
  m->val = calloc(capacity, sizeof(int));
  if (!m->busy || !m->keyp || !m->khash || !m->chain || !m->val) {
    lv_map_free(m);
    return 0;
  }
  m->cap = capacity;
  m->eq = eq;
  m->hash = hash;
  *out = m;
  return 1;
}

void lv_map_free(struct lv_map *m) {
  if (!m) return;
  free(m->busy);
  free(m->keyp);
  free(m->khash);
  free(m->chain);
  free(m->val);
  free(m);
}

/* map-impl-pow2.c:629-732 find_key: walk from hash&mask; a busy slot with the
 * same hash and an equal key is the hit; any other slot whose chain counter is
 * zero ends the search. */
static int map_find(struct lv_map *m, void *key, unsigned h) {
  unsigned mask = m->cap - 1;
  for (unsigned i = 0; i < m->cap; i++) {
    unsigned s = (h + i) & mask;
    if (m->busy[s] && m->khash[s] == h) {
      if (m->eq(m->keyp[s], key)) return (int)s;
    } else if (m->chain[s] == 0) {
      return -1;
    }
  }
  return -1;
}

int lv_map_get(struct lv_map *m, void *key, int *value_out) {
  unsigned h = m->hash(key); /* map.c:166 */
  int s = map_find(m, key, h);
  if (s < 0) return 0;
  *value_out = m->val[s];
  return 1;
}

/* map.c:180-206 + map-impl-pow2.c:1110-1217,2156-2222: the first free slot
 * from hash&mask; every busy slot passed on the way gains a chain count. */
void lv_map_put(struct lv_map *m, void *key, int value) {
  unsigned h = m->hash(key); /* hashed again, map.c:193 */
  unsigned mask = m->cap - 1;
  for (unsigned i = 0; i < m->cap; i++) {
    unsigned s = (h + i) & mask;
    if (!m->busy[s]) {
      m->busy[s] = 1;
      m->keyp[s] = key;
      m->khash[s] = h;
      m->val[s] = value;
      break;
    }
    m->chain[s] += 1;
  }
  m->size++;
}

/* map.c:238-273 + map-impl-pow2.c:790-972: walk to the key, decrementing the
 * chain counter of every slot before it, then clear the slot's busy bit. */
void lv_map_erase(struct lv_map *m, void *key, void **trash) {
  unsigned h = m->hash(key);
  unsigned mask = m->cap - 1;
  for (unsigned i = 0; i < m->cap; i++) {
    unsigned s = (h + i) & mask;
    if (m->busy[s] && m->khash[s] == h && m->eq(m->keyp[s], key)) {
      m->busy[s] = 0;
      *trash = m->keyp[s];
      break;
    }
    m->chain[s] -= 1;
  }
  m->size--;
}

unsigned lv_map_size(struct lv_map *m) { return m->size; }

/* --------------------------------------------------------------- dchain --
 * Index allocator + LRU list + timestamps (double-chain.c:16-19,
 * double-chain-impl.h:45-49). Cells 0 and 1 are the heads of the allocated
 * (doubly linked, LRU order) and free (singly linked, prev==next) lists;
 * index i lives in cell i+2.
 */
enum { DC_ALLOC = 0, DC_FREE = 1, DC_SHIFT = 2 };
struct dc_cell {
  int prev, next;
};
struct lv_dchain {
  struct dc_cell *cell;
  lv_time_t *ts;
  int range;
};

int lv_dchain_allocate(int index_range, struct lv_dchain **out) {
  struct lv_dchain *c = calloc(1, sizeof *c);
  if (!c) return 0;
  c->cell = malloc(sizeof(struct dc_cell) * (size_t)(index_range + DC_SHIFT));
  c->ts = calloc((size_t)index_range, sizeof(lv_time_t));
  if (!c->cell || !c->ts) {
    lv_dchain_free(c);
    return 0;
  }
  c->range = index_range;
  /* double-chain-impl.c:372-423: empty alloc list; free list 0,1,..,n-1 */
  c->cell[DC_ALLOC].prev = c->cell[DC_ALLOC].next = DC_ALLOC;
  c->cell[DC_FREE].prev = c->cell[DC_FREE].next = DC_SHIFT;
  for (int i = 0; i < index_range; i++) {
    int here = i + DC_SHIFT;
    int nxt = (i + 1 < index_range) ? here + 1 : DC_FREE;
    c->cell[here].prev = c->cell[here].next = nxt;
  }
  *out = c;
  return 1;
}

void lv_dchain_free(struct lv_dchain *c) {
  if (!c) return;
  free(c->cell);
  free(c->ts);
  free(c);
}

static void dc_append_alloc(struct lv_dchain *c, int cell) {
  struct dc_cell *head = &c->cell[DC_ALLOC];
  int tail = head->prev;
  c->cell[cell].next = DC_ALLOC;
  c->cell[cell].prev = tail;
  c->cell[tail].next = cell;
  head->prev = cell;
}

/* double-chain.c:350-392 + impl 1197-1415: pop the free-list head, append it
 * to the tail of the alloc list, stamp it. */
int lv_dchain_allocate_new_index(struct lv_dchain *c, int *index_out,
                                 lv_time_t t) {
  int cell = c->cell[DC_FREE].next;
  if (cell == DC_FREE) return 0;
  c->cell[DC_FREE].next = c->cell[DC_FREE].prev = c->cell[cell].next;
  dc_append_alloc(c, cell);
  *index_out = cell - DC_SHIFT;
  c->ts[*index_out] = t;
  return 1;
}

/* impl 2421-2479: a free cell has prev==next pointing into the free list
 * (never 0); an allocated cell either has prev!=next, or is the lone element
 * of the alloc list (prev==next==0). */
static int dc_is_alloc_cell(struct lv_dchain *c, int cell) {
  struct dc_cell *x = &c->cell[cell];
  if (x->prev != x->next) return 1;
  return x->next == DC_ALLOC;
}

/* double-chain.c:616-672 + impl 2191-2419: move to the alloc-list tail and
 * re-stamp; 0 (no-op) if the index is free. */
int lv_dchain_rejuvenate_index(struct lv_dchain *c, int index, lv_time_t t) {
  int cell = index + DC_SHIFT;
  struct dc_cell *x = &c->cell[cell];
  if (x->prev == x->next) {
    if (x->next != DC_ALLOC) return 0;
    c->ts[index] = t; /* only element: order unchanged, stamp updated */
    return 1;
  }
  c->cell[x->prev].next = x->next;
  c->cell[x->next].prev = x->prev;
  dc_append_alloc(c, cell);
  c->ts[index] = t;
  return 1;
}

/* impl 1839-2078: unlink from the alloc list and push onto the FRONT of the
 * free list (freed indices are reused first, LIFO). */
int lv_dchain_free_index(struct lv_dchain *c, int index) {
  int cell = index + DC_SHIFT;
  struct dc_cell *x = &c->cell[cell];
  if (x->prev == x->next && x->prev != DC_ALLOC) return 0;
  c->cell[x->prev].next = x->next;
  c->cell[x->next].prev = x->prev;
  x->next = x->prev = c->cell[DC_FREE].next;
  c->cell[DC_FREE].next = c->cell[DC_FREE].prev = cell;
  return 1;
}

/* double-chain.c:772-826: free the oldest index if its stamp is strictly
 * older than t. */
int lv_dchain_expire_one_index(struct lv_dchain *c, int *index_out,
                               lv_time_t t) {
  int oldest = c->cell[DC_ALLOC].next;
  if (oldest == DC_ALLOC) return 0;
  *index_out = oldest - DC_SHIFT;
  if (c->ts[*index_out] < t) return lv_dchain_free_index(c, *index_out);
  return 0;
}

int lv_dchain_is_index_allocated(struct lv_dchain *c, int index) {
  return dc_is_alloc_cell(c, index + DC_SHIFT);
}

int lv_dchain_dump(struct lv_dchain *c, int index_range, int *alloc_order,
                   int *n_alloc, int *free_order, int *n_free, lv_time_t *ts) {
  int k = 0;
  for (int x = c->cell[DC_ALLOC].next; x != DC_ALLOC && k < index_range;
       x = c->cell[x].next)
    alloc_order[k++] = x - DC_SHIFT;
  *n_alloc = k;
  k = 0;
  for (int x = c->cell[DC_FREE].next; x != DC_FREE && k < index_range;
       x = c->cell[x].next)
    free_order[k++] = x - DC_SHIFT;
  *n_free = k;
  for (int i = 0; i < index_range; i++) ts[i] = c->ts[i];
  return 1;
}

/* --------------------------------------------------------------- vector --
 * vector.c:147-311: fixed-size element array, every element initialised. */
struct lv_vector {
  char *data;
  int elem;
  unsigned cap;
};

int lv_vector_allocate(int elem_size, unsigned capacity, lv_init_fn *init,
                       struct lv_vector **out) {
  struct lv_vector *v = calloc(1, sizeof *v);
  if (!v) return 0;
  v->data = malloc((size_t)elem_size * capacity);
  if (!v->data) {
    free(v);
    return 0;
  }
  v->elem = elem_size;
  v->cap = capacity;
  for (unsigned i = 0; i < capacity; i++) init(v->data + (size_t)elem_size * i);
  *out = v;
  return 1;
}
void lv_vector_borrow(struct lv_vector *v, int index, void **val_out) {
  *val_out = v->data + (ptrdiff_t)index * v->elem;
}
void lv_vector_return(struct lv_vector *v, int index, void *val) {
  (void)v;
  (void)index;
  (void)val;
}
void lv_vector_free(struct lv_vector *v) {
  if (!v) return;
  free(v->data);
  free(v);
}

/* ------------------------------------------------------------ expirator --
 * expirator.c:110-218: while the oldest index is expired, free it and erase
 * its key (found through the key vector) from the map. */
int lv_expire_items_single_map(struct lv_dchain *c, struct lv_vector *v,
                               struct lv_map *m, lv_time_t t) {
  int n = 0, idx = -1;
  while (lv_dchain_expire_one_index(c, &idx, t)) {
    void *key;
    lv_vector_borrow(v, idx, &key);
    lv_map_erase(m, key, &key);
    lv_vector_return(v, idx, key);
    n++;
  }
  return n;
}

/* ------------------------------------------------------------------ cht --
 * cht.c:546-877 cht_fill_cht. Backend i visits buckets in the order
 * (31*i mod h) + ((i mod (h-1)) + 1) * j  (mod h), j = 0..h-1. Each bucket's
 * priority list is filled, in rounds j = 0..h-1, by backends 0..cap-1
 * whose j-th visit lands on it. Table layout: cht[bucket*cap + priority]. */
int lv_cht_fill_cht(struct lv_vector *cht, uint32_t height,
                    uint32_t backend_capacity) {
  uint64_t n = (uint64_t)height * backend_capacity;
  uint32_t *perm = malloc(sizeof(uint32_t) * n);
  uint32_t *fill = calloc(height, sizeof(uint32_t));
  if (!perm || !fill) {
    free(perm);
    free(fill);
    return 0;
  }
  for (uint32_t b = 0; b < backend_capacity; b++) {
    uint64_t off = (uint64_t)(uint32_t)(b * 31u) % height;
    uint64_t step = (uint64_t)b % (height - 1) + 1;
    for (uint32_t j = 0; j < height; j++)
      perm[(uint64_t)b * height + j] = (uint32_t)((off + step * j) % height);
  }
  for (uint32_t j = 0; j < height; j++) {
    for (uint32_t b = 0; b < backend_capacity; b++) {
      uint32_t bucket = perm[(uint64_t)b * height + j];
      uint32_t prio = fill[bucket]++;
      void *slot;
      lv_vector_borrow(cht, (int)(backend_capacity * bucket + prio), &slot);
      *(uint32_t *)slot = b;
    }
  }
  free(perm);
  free(fill);
  return 1;
}

/* cht.c:969-1062: scan bucket (hash mod h) in priority order for the first
 * backend index that is currently allocated in `active`. */
int lv_cht_find_preferred_available_backend(uint64_t hash,
                                            struct lv_vector *cht,
                                            struct lv_dchain *active,
                                            uint32_t height,
                                            uint32_t backend_capacity,
                                            int *chosen) {
  uint64_t bucket = hash % height;
  for (uint32_t p = 0; p < backend_capacity; p++) {
    void *slot;
    lv_vector_borrow(cht, (int)(bucket * backend_capacity + p), &slot);
    uint32_t cand = *(uint32_t *)slot;
    if (lv_dchain_is_index_allocated(active, (int)cand)) {
      *chosen = (int)cand;
      return 1;
    }
  }
  return 0;
}
