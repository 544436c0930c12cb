/* Plain-C client of include/zero_amd.h (host-only entry points, no GPU needed): proves the
 * header is valid C99 and the library links and answers from C, the way a cgo / FFI binding
 * would use it.  Built and run by tests/test_abi.py::test_plain_c_client. */
#include <stdio.h>
#include <string.h>

#include "zero_amd.h"

#define CHECK(cond)                                                   \
  do {                                                                \
    if (!(cond)) {                                                    \
      fprintf(stderr, "FAIL %s:%d: %s (%s)\n", __FILE__, __LINE__, #cond, \
              zs_last_error());                                       \
      return 1;                                                       \
    }                                                                 \
  } while (0)

int main(void) {
  CHECK(zs_abi_version() == ZS_ABI_VERSION);
  /* the reference MLP: 6 x Linear(D, D) = 12 tensors, W then b (zero1.py:113-120) */
  int64_t numels[12];
  for (int i = 0; i < 12; ++i) numels[i] = (i % 2 == 0) ? 64 * 64 : 64;
  zs_plan* plan = NULL;
  CHECK(zs_plan_create_ex(12, numels, NULL, 8, 3, ZS_LAYOUT_R, 64, 256, ZS_BUCKETS_RAGGED, &plan) ==
        ZS_OK);
  /* SURVEY.md §8(b)'s literal form: 64 KiB buckets (fp32 bytes) over 8 ranks */
  zs_plan* lit = NULL;
  CHECK(zs_plan_create(12, numels, NULL, 8, 3, ZS_LAYOUT_R, 64 << 10, &lit) == ZS_OK);
  int64_t ls = -1, le = -1;
  CHECK(zs_plan_owner_range(lit, 3, &ls, &le) == ZS_OK && ls == 6 && le == 8);
  CHECK(zs_plan_destroy(lit) == ZS_OK);
  /* ws = 8, n = 12: ranges [0,2),[2,4),[4,6),[6,8),[8],[9],[10],[11] */
  int64_t s = -1, e = -1;
  CHECK(zs_plan_owner_range(plan, 3, &s, &e) == ZS_OK && s == 6 && e == 8);
  CHECK(zs_plan_owner_range(plan, 7, &s, &e) == ZS_OK && s == 11 && e == 12);
  int owner = -1;
  CHECK(zs_plan_owner_of(plan, 9, &owner) == ZS_OK && owner == 5);
  int64_t k = 0, total = 0;
  CHECK(zs_plan_num_buckets(plan, &k) == ZS_OK && k > 0);
  for (int64_t b = 0; b < k; ++b) {
    int64_t bytes = 0, nseg = 0;
    CHECK(zs_plan_bucket_bytes(plan, b, ZS_BF16, &bytes) == ZS_OK && bytes > 0);
    CHECK(zs_plan_num_segments(plan, b, &nseg) == ZS_OK);
    int64_t param[64], rank[64], poff[64], boff[64], len[64];
    CHECK(nseg <= 64);
    CHECK(zs_plan_segments(plan, b, param, rank, poff, boff, len) == ZS_OK);
    for (int64_t j = 0; j < nseg; ++j) {
      CHECK(2 * (boff[j] + len[j]) <= bytes);
      total += len[j];
    }
  }
  CHECK(total == 6 * (64 * 64 + 64)); /* every element of every param lands in one bucket */
  /* errors come back as codes with a message, never as a crash */
  CHECK(zs_plan_bucket_bytes(plan, k, ZS_BF16, &total) == ZS_ERR_INVALID);
  CHECK(strstr(zs_last_error(), "out of range") != NULL);
  CHECK(zs_adam_step_ex(NULL, NULL, NULL, ZS_F32, NULL, NULL, 16, 1e-3, 0.9, 0.999, 1e-8, 0.0, 0, 1,
                        1.0, NULL, 0.0, 0) == ZS_ERR_INVALID);
  CHECK(zs_adam_step(NULL, NULL, NULL, ZS_F32, NULL, NULL, 16, 1e-3f, 0.9f, 0.999f, 1e-8f, 0.0f, 0, 1,
                     0.125f, NULL, 0.0f, 0) == ZS_ERR_INVALID);
  CHECK(zs_range_push("optimizer_step") == ZS_OK && zs_range_pop() == ZS_OK);
  CHECK(zs_plan_destroy(plan) == ZS_OK);
  printf("c-abi ok: %lld buckets\n", (long long)k);
  return 0;
}
