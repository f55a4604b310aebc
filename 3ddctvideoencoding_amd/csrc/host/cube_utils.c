/* cube_utils.c -- diagonal-slice ordering (CubeUtils.c:5-46 / CubeUtils.java:7-41 semantics). */
#include "cube_utils.h"

#include <stdlib.h>

static int imin(int a, int b) { return a < b ? a : b; }

struct SlicesPositions *cubeUtils_diagonalSlices(int width, int height, int depth) {
    if (width <= 0 || height <= 0 || depth <= 0) return NULL;
    struct SlicesPositions *sp = (struct SlicesPositions *)malloc(sizeof(*sp));
    if (!sp) return NULL;
    sp->length = width * height * depth;
    sp->positions = (struct ThreeDimensionalCoordinates *)malloc(sizeof(struct ThreeDimensionalCoordinates) * sp->length);
    if (!sp->positions) {
        free(sp);
        return NULL;
    }
    int n = 0;
    const int maxSum = (width - 1) + (height - 1) + (depth - 1);
    for (int t = 0; t <= maxSum; t++) {
        /* every (x, y, z) with x + y + z == t; y outer, z middle, x inner */
        const int yHi = imin(height - 1, t), zHi = imin(depth - 1, t);
        for (int y = 0; y <= yHi; y++)
            for (int z = 0; z <= zHi; z++) {
                const int x = t - y - z;
                if (x < 0 || x > width - 1) continue;
                sp->positions[n].x = x;
                sp->positions[n].y = y;
                sp->positions[n].z = z;
                n++;
            }
    }
    return sp;
}

void cubeUtils_deallocatePositions(struct SlicesPositions *sp) {
    if (!sp) return;
    free(sp->positions);
    free(sp);
}
