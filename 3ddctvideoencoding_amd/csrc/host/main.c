/* main.c -- CLI with the reference's argument convention (main.c:5-49):
 *   dct3d_codec list_devices
 *   dct3d_codec encode|decode <input> <output> <width> <height> <frames> [device_index (1-based)] [block_depth 8|4]
 * (list_platforms is accepted as an alias of list_devices.)  device_index may be a comma-separated list
 * ("1,2,3"): encode_multi / decode_multi over those devices. */
#include <errno.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "codec.h"
#include "dct3d.h"

static void usage(void) {
    printf("Usage\n\n");
    printf("dct3d_codec list_devices -> List available HIP devices\n");
    printf("dct3d_codec encode|decode <input file> <output file> <width> <height> <nr of frames> "
           "<device_index (optional, 1-based; a list a,b,... uses several)> <block depth 8|4 (optional)> -> "
           "Encode/Decode given file\n");
}

/* "1" or "1,2,3": 1-based device numbers (the reference's platformIndex, main.c:33-37).  Every entry must
 * be a positive decimal number; an empty entry, trailing junk, a value <= 0 or more than max entries is
 * an error (non-zero return). */
static int parse_devices(const char *arg, int *devs, int max, int *n) {
    *n = 0;
    const char *p = arg;
    for (;;) {
        char *end = NULL;
        errno = 0;
        const long v = strtol(p, &end, 10);
        if (end == p || errno || v <= 0 || v > 1 << 20 || *n >= max) return -1;
        devs[(*n)++] = (int)v;
        if (*end == '\0') return 0;
        if (*end != ',') return -1;
        p = end + 1;
    }
}

int main(int argc, char *argv[]) {
    if (argc < 2) {
        usage();
        return 0;
    }
    if (!strcmp(argv[1], "list_devices") || !strcmp(argv[1], "list_platforms")) {
        for (int d = 0;; d++) {
            dct3d_ctx *c = NULL;
            if (dct3d_ctx_create(d, 8, 8, 8, &c)) {
                if (d == 0) printf("No HIP device available\n");
                break;
            }
            printf("%d - HIP device %d\n", d + 1, d);
            dct3d_ctx_destroy(c);
        }
        return 0;
    }
    if (argc < 7) {
        usage();
        return 1;
    }
    const int width = atoi(argv[4]), height = atoi(argv[5]), frames = atoi(argv[6]);
    int devs[64], n_dev = 0;
    if (argc > 7 && parse_devices(argv[7], devs, 64, &n_dev)) {
        printf("Invalid device list '%s': 1-based device numbers, comma-separated, at most 64\n", argv[7]);
        usage();
        return 1;
    }
    if (n_dev == 0) devs[n_dev++] = 1;
    const int depth = argc > 8 ? atoi(argv[8]) : DCT_BLOCK_DEPTH;
    if (!strcmp(argv[1], "encode"))
        return n_dev > 1 ? encode_multi(argv[2], argv[3], width, height, frames, devs, n_dev, depth, 0)
                         : encode_ex(argv[2], argv[3], width, height, frames, devs[0], depth, 0);
    if (!strcmp(argv[1], "decode"))
        return n_dev > 1 ? decode_multi(argv[2], argv[3], width, height, frames, devs, n_dev, depth, 0)
                         : decode_ex(argv[2], argv[3], width, height, frames, devs[0], depth, 0);
    usage();
    return 1;
}
