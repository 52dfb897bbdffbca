/* Host-only sanitizer harness for csrc/host/jpeg_entropy.c: decodes every file
 * named on the command line (seeded corruptions written by
 * tools/jpeg_fuzz_asan.sh) under AddressSanitizer + UBSan.  A read or write
 * outside the input, table or coefficient buffers aborts with a report. */
#include <stdio.h>
#include <stdlib.h>
#include "hkp_jpeg.h"

int main(int argc, char** argv) {
    int ok = 0, bad = 0;
    for (int i = 1; i < argc; ++i) {
        FILE* f = fopen(argv[i], "rb");
        if (!f) return 2;
        fseek(f, 0, SEEK_END);
        long n = ftell(f);
        fseek(f, 0, SEEK_SET);
        uint8_t* buf = (uint8_t*)malloc((size_t)n);   /* exact size: ASan sees any over-read */
        if (fread(buf, 1, (size_t)n, f) != (size_t)n) return 2;
        fclose(f);
        hkpj_geom g;
        int rc = hkpj_probe(buf, n, &g);
        if (rc == HKPJ_OK) {
            int16_t* coefs = (int16_t*)malloc((size_t)g.nblocks * 64 * sizeof(int16_t));
            uint16_t* qt = (uint16_t*)malloc((size_t)g.ncomp * 64 * sizeof(uint16_t));
            rc = hkpj_decode(buf, n, &g, coefs, qt);
            free(coefs);
            free(qt);
        }
        rc == HKPJ_OK ? ++ok : ++bad;
        free(buf);
    }
    printf("decoded %d, rejected %d\n", ok, bad);
    return 0;
}
