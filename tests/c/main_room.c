/*
 * The reference's console harness (KernelFolder/Kernel/Kernel.cu:1003-1217) restated as a plain C
 * caller of libmhgpu.so: the same room (:1007-1166), the same gpuConfig (:1187-1194) and the same
 * KernelWrapper call (:1198), through include/mh_kernel.h only -- what a C caller of the
 * reference DLL compiles and links. Differences from main(), each because the reference's line
 * has no counterpart in this library or needs a person at the console:
 *   - no basicCudaDeviceInformation (:1005, a CUDA device query through helper_cuda.h);
 *   - WeightOffLimits is set to 0 (main() leaves it uninitialised; it never enters totalCosts);
 *   - no scanf wait (:1215-1216);
 *   - argv[1] optionally overrides gpuCfg.gridxDim (main() runs 1 chain), and every point and
 *     cost is printed as a hex float (%a) so tests/test_c_harness.py can compare bits.
 * The seed comes from $MH_SEED (KernelWrapper's documented behaviour; time(NULL) otherwise).
 */
#include <stdio.h>
#include <stdbool.h>
#include <stdlib.h>

#include "mh_kernel.h"

#define PI 3.1416

int main(int argc, char** argv) {
    enum { N = 32, NRel = 1, NClearances = 2 };
    Surface srf;
    srf.nObjs = N;
    srf.nRelationships = NRel;
    srf.nClearances = NClearances;
    srf.WeightFocalPoint = -2.0f;
    srf.WeightPairWise = -2.0f;
    srf.WeightVisualBalance = 1.5f;
    srf.WeightSymmetry = -2.0f;
    srf.WeightOffLimits = 0.0f;
    srf.WeightClearance = -2.0f;
    srf.WeightSurfaceArea = -2.0f;
    srf.centroidX = 0.0;
    srf.centroidY = 0.0;
    srf.focalX = 5.0;
    srf.focalY = 5.0;
    srf.focalRot = 0.0;

    vertex surfaceRectangle[4] = {{10, 10, 0}, {10, 0, 0}, {0, 0, 0}, {0, 10, 0}};
    /* clearance shapes (vtx 0-7), then off-limits shapes (8-15), Kernel.cu:1044-1109 */
    vertex vtx[16] = {{2, 2, 0}, {2, 0, 0}, {0, 0, 0}, {0, 2, 0},
                      {3, 2, 0}, {3, 0, 0}, {1, 0, 0}, {1, 2, 0},
                      {2, 2, 0}, {2, 0, 0}, {0, 0, 0}, {0, 2, 0},
                      {3, 2, 0}, {3, 0, 0}, {1, 0, 0}, {1, 2, 0}};
    rectangle clearances[NClearances] = {{0, 1, 2, 3, 0}, {4, 5, 6, 7, 1}};
    rectangle offlimits[N];
    positionAndRotation cfg[N];
    for (int i = 0; i < N; i++) {
        const rectangle even = {8, 9, 10, 11, 0}, odd = {12, 13, 14, 15, 1};
        offlimits[i] = (i % 2 == 0) ? even : odd;
        cfg[i].x = i * 2.0;
        cfg[i].y = i * 2.0;
        cfg[i].z = 0.0;
        cfg[i].rotX = 0.0;
        cfg[i].rotY = 0.0;
        cfg[i].rotZ = 0.0;
        cfg[i].frozen = false;
        cfg[i].length = 1.0;
        cfg[i].width = 1.0;
    }
    relationshipStruct rss[NRel];
    rss[0].TargetRange.targetRangeStart = 2.0;
    rss[0].TargetRange.targetRangeEnd = 4.0;
    rss[0].DegreesOfAtrraction = 2.0;
    rss[0].SourceIndex = 0;
    rss[0].TargetIndex = 1;
    relationshipAngleStruct rsa[NRel];
    rsa[0].angleMin = PI / 4;
    rsa[0].angleMax = 5 * PI / 8;
    rsa[0].SourceIndex = 0;
    rsa[0].TargetIndex = 1;
    printf("Target angles are (%f,%f)\n", rsa[0].angleMin, rsa[0].angleMax);

    gpuConfig gpuCfg;
    gpuCfg.gridxDim = argc > 1 ? atoi(argv[1]) : 1;
    gpuCfg.gridyDim = 0;
    gpuCfg.blockxDim = 64;
    gpuCfg.blockyDim = 0;
    gpuCfg.blockzDim = 0;
    gpuCfg.iterations = 100;

    result* res = KernelWrapper(rss, rsa, cfg, clearances, offlimits, vtx, surfaceRectangle, &srf,
                                &gpuCfg);
    if (!res) {
        fprintf(stderr, "KernelWrapper failed: %s\n", KernelLastError());
        return EXIT_FAILURE;
    }
    printf("Results:\n");
    for (int i = 0; i < gpuCfg.gridxDim; i++) {
        printf("Result %d costs %a %a %a %a %a %a %a %a\n", i, res[i].costs.totalCosts,
               res[i].costs.PairWiseCosts, res[i].costs.VisualBalanceCosts,
               res[i].costs.FocalPointCosts, res[i].costs.SymmetryCosts,
               res[i].costs.ClearanceCosts, res[i].costs.OffLimitsCosts,
               res[i].costs.SurfaceAreaCosts);
        for (int j = 0; j < srf.nObjs; j++)
            printf("Point [%d] %a %a %a %a %a %a\n", j, res[i].points[j].x, res[i].points[j].y,
                   res[i].points[j].z, res[i].points[j].rotX, res[i].points[j].rotY,
                   res[i].points[j].rotZ);
    }
    KernelFreeResult(res);
    return EXIT_SUCCESS;
}
