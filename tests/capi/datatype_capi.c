/* Derived datatypes through the C API (reference parsec/datatype.h:14-130:
 * contiguous, vector, hvector, indexed, struct, resized): sizes, extents and
 * pack/unpack round trips checked against hand-computed layouts. */
#include <stddef.h>
#include <stdio.h>
#include <string.h>

#include "parsec.h"

static int fails = 0;
#define CHECK(c, msg)                                   \
    do {                                                \
        if (!(c)) {                                     \
            fprintf(stderr, "FAIL line %d: %s\n", __LINE__, msg); \
            fails++;                                    \
        }                                               \
    } while (0)

int main(void) {
    double src[64], packed[64], back[64];
    int i, size;
    ptrdiff_t lb, ext;
    for (i = 0; i < 64; i++) src[i] = (double)(i + 1);

    /* vector: 4 blocks of 2 doubles, stride 8 */
    parsec_datatype_t vec;
    parsec_type_create_vector(4, 2, 8, parsec_datatype_double_t, &vec);
    parsec_type_size(vec, &size);
    parsec_type_extent(vec, &lb, &ext);
    CHECK(size == 8 * 8 && ext == (3 * 8 + 2) * 8 && lb == 0, "vector size/extent");
    parsec_type_pack(vec, src, packed);
    CHECK(packed[0] == 1 && packed[1] == 2 && packed[2] == 9 && packed[7] == 26, "vector pack");

    /* hvector of the vector: 2 of them, 256 bytes apart */
    parsec_datatype_t hv;
    parsec_type_create_hvector(2, 1, 256, vec, &hv);
    parsec_type_size(hv, &size);
    CHECK(size == 2 * 64, "hvector size");
    parsec_type_pack(hv, src, packed);
    CHECK(packed[8] == src[32] && packed[15] == src[32 + 25], "hvector pack");

    /* indexed doubles: {3 at 1, 2 at 10} */
    int bl[2] = {3, 2}, dp[2] = {1, 10};
    parsec_datatype_t idx;
    parsec_type_create_indexed(2, bl, dp, parsec_datatype_double_t, &idx);
    parsec_type_size(idx, &size);
    parsec_type_extent(idx, &lb, &ext);
    CHECK(size == 5 * 8 && ext == 12 * 8, "indexed size/extent");
    parsec_type_pack(idx, src, packed);
    CHECK(packed[0] == 2 && packed[2] == 4 && packed[3] == 11 && packed[4] == 12, "indexed pack");

    /* struct { int32 a; double b[2]; } laid out at byte 0 / 8 */
    struct rec { int a; double b[2]; } recs[2] = {{7, {1.5, 2.5}}, {9, {3.5, 4.5}}}, rback[2];
    int sbl[2] = {1, 2};
    ptrdiff_t sdp[2] = {offsetof(struct rec, a), offsetof(struct rec, b)};
    parsec_datatype_t sty[2] = {parsec_datatype_int32_t, parsec_datatype_double_t};
    parsec_datatype_t st, st_r;
    parsec_type_create_struct(2, sbl, sdp, sty, &st);
    parsec_type_size(st, &size);
    CHECK(size == 4 + 16, "struct size");
    /* resized to the C struct's extent so two records pack back to back */
    parsec_type_create_resized(st, 0, sizeof(struct rec), &st_r);
    parsec_type_extent(st_r, &lb, &ext);
    CHECK(ext == (ptrdiff_t)sizeof(struct rec), "resized extent");
    unsigned char buf[64];
    parsec_type_pack(st_r, &recs[0], buf);
    memset(rback, 0, sizeof(rback));
    parsec_type_unpack(st_r, buf, &rback[0]);
    CHECK(rback[0].a == 7 && rback[0].b[0] == 1.5 && rback[0].b[1] == 2.5, "struct round trip");
    int a2;
    memcpy(&a2, buf, 4);
    CHECK(a2 == 7, "struct packed int first");

    /* round trip of the vector leaves the gaps untouched */
    memset(back, 0, sizeof(back));
    parsec_type_pack(vec, src, packed);
    parsec_type_unpack(vec, packed, back);
    CHECK(back[0] == 1 && back[2] == 0 && back[8] == 9 && back[25] == 26 && back[26] == 0, "vector round trip");

    /* lower triangle of a 4x4 tile */
    parsec_datatype_t low;
    parsec_type_create_lower(4, 4, 1, parsec_datatype_double_t, &low);
    parsec_type_size(low, &size);
    CHECK(size == 10 * 8, "lower size");

    if (fails) { printf("datatype failures %d\n", fails); return 1; }
    printf("datatype ok\n");
    return 0;
}
