/* main.c -- CLI with the reference's argument convention (main.c:5-49):
 *   dct3d_codec list_devices
 *   dct3d_codec encode|decode <input> <output> <width> <height> <frames> [device_index (1-based)] [block_depth 8|4]
 * (list_platforms is accepted as an alias of list_devices.) */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "codec.h"
#include "dct3d.h"

static void usage(void) {
    printf("Usage\n\n");
    printf("dct3d_codec list_devices -> List available HIP devices\n");
    printf("dct3d_codec encode|decode <input file> <output file> <width> <height> <nr of frames> "
           "<device_index (optional, 1-based)> <block depth 8|4 (optional)> -> Encode/Decode given file\n");
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
    const int dev = argc > 7 ? atoi(argv[7]) : 1;
    const int depth = argc > 8 ? atoi(argv[8]) : DCT_BLOCK_DEPTH;
    if (!strcmp(argv[1], "encode")) return encode_ex(argv[2], argv[3], width, height, frames, dev, depth, 0);
    if (!strcmp(argv[1], "decode")) return decode_ex(argv[2], argv[3], width, height, frames, dev, depth, 0);
    usage();
    return 1;
}
