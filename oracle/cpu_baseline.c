/*
 * cpu_baseline.c -- multi-core driver of the oracle for bench.py's cpu_baseline leg.
 * TEST / MEASUREMENT INFRASTRUCTURE ONLY (see ipxg_oracle.h): nothing in the product loads it.
 *
 * It runs the reference's parallel shape on the host: one pipeline per core, each an
 * independent parse_packet + NHTFlowCache::put_pkt loop over its own pre-loaded slice of the
 * packets, with a private cache (ipfixprobe.cpp:381-464 builds one input thread + one cache
 * per input queue; the NIC's symmetric RSS keeps both directions of a biflow in one queue,
 * dpdkDevice.cpp:230-262).  The slices are made by the caller (not timed).  Each thread is
 * pinned to one CPU of the process's affinity set; the threads start together once every
 * cache is built, and the wall time runs from that start to the last thread's finish() (the
 * reference drains its cache at end of input, workers.cpp:136, cache.cpp:276-288).
 */
#define _GNU_SOURCE
#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ipxg_oracle.h"

typedef struct {
    const uint8_t* arena;
    const ipxg_pkt_desc* desc;
    size_t n;
    uint32_t datalink;
    uint32_t cache_exp;
    int cpu; /* -1: not pinned */
    volatile int* go;
    int* ready;
    double t_end;
    uint64_t records, no_res;
    int err;
} shard_job;

static double now_s(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (double)ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void* shard_main(void* arg)
{
    shard_job* j = (shard_job*)arg;
    if (j->cpu >= 0) {
        cpu_set_t set;
        CPU_ZERO(&set);
        CPU_SET(j->cpu, &set);
        pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
    }
    /* the cache is built before the clock starts, as the reference builds its storage
     * plugin at start-up (ipfixprobe.cpp:414-421) */
    oracle_cache* c = oracle_cache_new(j->cache_exp, 4, 300, 30, 0, 1, 10007, 3);
    __atomic_add_fetch(j->ready, 1, __ATOMIC_SEQ_CST);
    while (!__atomic_load_n(j->go, __ATOMIC_ACQUIRE)) {
    }
    if (!c) {
        j->err = 1;
        j->t_end = now_s();
        return NULL;
    }
    oracle_cache_run(c, j->arena, j->desc, j->n, j->datalink);
    oracle_cache_finish(c);
    ipxg_stats st;
    oracle_cache_stats(c, &st);
    j->records = oracle_cache_pending(c);
    j->no_res = st.end_no_res;
    j->t_end = now_s();
    oracle_cache_free(c);
    return NULL;
}

/*
 * Run nshards pipelines, shard k over desc[first[k] .. first[k] + count[k]) (descriptors
 * grouped by shard by the caller), thread k pinned to cpus[k] (cpus may be NULL).
 * Returns the wall time in seconds (< 0 on failure); records / NO_RES exports summed.
 */
double oracle_bench_mt(const uint8_t* arena, const ipxg_pkt_desc* desc, const uint64_t* first,
                       const uint64_t* count, int nshards, const int* cpus, uint32_t cache_exp,
                       uint32_t datalink, uint64_t* records, uint64_t* no_res)
{
    if (nshards < 1) return -1.0;
    shard_job* jobs = (shard_job*)calloc((size_t)nshards, sizeof(shard_job));
    pthread_t* th = (pthread_t*)calloc((size_t)nshards, sizeof(pthread_t));
    volatile int go = 0;
    int ready = 0;
    if (!jobs || !th) {
        free(jobs);
        free(th);
        return -1.0;
    }
    int started = 0;
    for (int k = 0; k < nshards; ++k) {
        jobs[k].arena = arena;
        jobs[k].desc = desc + first[k];
        jobs[k].n = count[k];
        jobs[k].datalink = datalink;
        jobs[k].cache_exp = cache_exp;
        jobs[k].cpu = cpus ? cpus[k] : -1;
        jobs[k].go = &go;
        jobs[k].ready = &ready;
        if (pthread_create(&th[k], NULL, shard_main, &jobs[k]) != 0) break;
        started++;
    }
    /* start line: every started thread has built its cache */
    while (__atomic_load_n(&ready, __ATOMIC_ACQUIRE) < started) {
    }
    const double t0 = now_s();
    __atomic_store_n(&go, 1, __ATOMIC_RELEASE);
    for (int k = 0; k < started; ++k) pthread_join(th[k], NULL);
    double t1 = t0;
    uint64_t rec = 0, nr = 0;
    int err = started < nshards;
    for (int k = 0; k < started; ++k) {
        if (jobs[k].t_end > t1) t1 = jobs[k].t_end;
        rec += jobs[k].records;
        nr += jobs[k].no_res;
        err |= jobs[k].err;
    }
    free(jobs);
    free(th);
    if (records) *records = rec;
    if (no_res) *no_res = nr;
    return err ? -1.0 : t1 - t0;
}
