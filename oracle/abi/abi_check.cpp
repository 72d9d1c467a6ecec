// abi_check: compares the two layout tables; prints every mismatch, exit 1
// if any.  Test infrastructure (tests/test_ref_pinning.py).
#include <stdio.h>
#include <string.h>
#include <stddef.h>
#include "abi_fields.h"
extern const AbiEntry abi_ref[];
extern const AbiEntry abi_ours[];
int main() {
    int bad = 0, n = 0;
    for (; abi_ref[n].type; ++n) {
        const AbiEntry &r = abi_ref[n], &o = abi_ours[n];
        if (r.value != o.value) {
            printf("MISMATCH %s.%s ref %zu ours %zu\n", r.type, r.field, r.value, o.value);
            ++bad;
        }
    }
    printf("%d entries, %d mismatches\n", n, bad);
    return bad ? 1 : 0;
}
