/*
 * cube_utils.h -- diagonal-slice ordering of a cube's coefficients
 * (replaces 3d-DCT-video-encoding-OpenCL/CubeUtils.h:11-24; Java CubeUtils.java:7-41).
 * Positions are ordered by x+y+z ascending; within a slice y outer, z middle, x inner.
 */
#ifndef DCT3D_CUBE_UTILS_H_
#define DCT3D_CUBE_UTILS_H_

#ifdef __cplusplus
extern "C" {
#endif

struct ThreeDimensionalCoordinates {
    int x;
    int y;
    int z;
};

struct SlicesPositions {
    struct ThreeDimensionalCoordinates *positions;
    int length;
};

struct SlicesPositions *cubeUtils_diagonalSlices(int width, int height, int depth);
void cubeUtils_deallocatePositions(struct SlicesPositions *slicesPositions);

#ifdef __cplusplus
}
#endif

#endif
