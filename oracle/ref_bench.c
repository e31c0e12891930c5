/*
 * ORACLE -- test/bench infrastructure only (never linked into the product).
 *
 * Multi-core driver for the reference's own message_passing() (message_passing.c:7-82),
 * linked against that file compiled unchanged from /root/reference by `make -C oracle ref`
 * into _ref/ref_bench.so.  bench.py times it as the "reference" CPU baseline of the BEC hot
 * path: one word per call as parallel_simulator.py:131-166 does, words spread over
 * OpenMP threads (the reference itself parallelises with processes,
 * parallel_simulator.py:403-445).
 */
#include <omp.h>
#include <stdlib.h>
#include <string.h>

int message_passing(int *Mvc, int iterations, int *variable_to_check_list, int *check_to_variable_list,
                    int *errors, int n, int k, int dv, int dc);

/* words: B x n int32 (0/1/2, consumed in place); errors: B x iterations int32 (zeroed here);
   its: B.  Returns the thread count used. */
int ref_bench_message_passing(int *words, int B, int iterations, int *v2c, int *c2v, int *errors, int *its,
                              int n, int k, int dv, int dc, int threads)
{
    if (threads < 1) threads = 1;
    int used = 1;
#pragma omp parallel num_threads(threads)
    {
#pragma omp single
        used = omp_get_num_threads();
#pragma omp for schedule(dynamic, 4)
        for (int b = 0; b < B; b++) {
            int *e = errors + (size_t)b * iterations;
            memset(e, 0, sizeof(int) * (size_t)iterations);
            its[b] = message_passing(words + (size_t)b * n, iterations, v2c, c2v, e, n, k, dv, dc);
        }
    }
    return used;
}
