/*
 * CPU baseline harness — ORACLE / BENCH-ONLY (bench.py's cpu_baseline leg).
 *
 * Times the reference's own verifier: libsodium 1.0.18 crypto_sign_open (what
 * stp_core/crypto/nacl_wrappers.py:108 reaches through libnacl), dlopen'ed from the image, on
 * `threads` pthreads over the same (sm, pk) records the GPU verifies. If libsodium is absent the
 * caller times the C oracle (ed25519_oracle.c) instead and labels it a port.
 * Returns the number of accepted records (so callers can check the verdicts agree), or -1.
 */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

typedef int (*open_fn)(unsigned char*, unsigned long long*, const unsigned char*, unsigned long long,
                       const unsigned char*);
typedef int (*init_fn)(void);

int oracle_sign_open(const uint8_t* sm, size_t smlen, const uint8_t pk[32]);

struct job {
    const uint8_t* blob;
    const uint64_t* off;
    const uint8_t* pk;
    uint64_t lo, hi;
    open_fn fn;
    uint64_t accepted;
};

static void* worker(void* arg) {
    struct job* j = (struct job*)arg;
    uint64_t maxlen = 0;
    for (uint64_t i = j->lo; i < j->hi; i++)
        if (j->off[i + 1] - j->off[i] > maxlen) maxlen = j->off[i + 1] - j->off[i];
    unsigned char* m = (unsigned char*)malloc(maxlen + 64);
    for (uint64_t i = j->lo; i < j->hi; i++) {
        const uint64_t len = j->off[i + 1] - j->off[i];
        int rc;
        if (j->fn) {
            unsigned long long mlen = 0;
            rc = j->fn(m, &mlen, j->blob + j->off[i], len, j->pk + 32 * i);
        } else {
            rc = oracle_sign_open(j->blob + j->off[i], len, j->pk + 32 * i);
        }
        j->accepted += rc == 0;
    }
    free(m);
    return NULL;
}

/* use_sodium: 1 = libsodium at `path`, 0 = the C oracle */
int64_t cpu_baseline_run(const char* path, int use_sodium, const uint8_t* blob, const uint64_t* off,
                         const uint8_t* pk, uint64_t n, int threads) {
    open_fn fn = NULL;
    if (use_sodium) {
        void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
        if (!h) return -1;
        init_fn init = (init_fn)dlsym(h, "sodium_init");
        fn = (open_fn)dlsym(h, "crypto_sign_open");
        if (!init || !fn || init() < 0) return -1;
    }
    if (threads < 1) threads = 1;
    pthread_t* tid = (pthread_t*)calloc(threads, sizeof(pthread_t));
    struct job* jobs = (struct job*)calloc(threads, sizeof(struct job));
    for (int t = 0; t < threads; t++) {
        jobs[t].blob = blob;
        jobs[t].off = off;
        jobs[t].pk = pk;
        jobs[t].lo = n * t / threads;
        jobs[t].hi = n * (t + 1) / threads;
        jobs[t].fn = fn;
        pthread_create(&tid[t], NULL, worker, &jobs[t]);
    }
    uint64_t acc = 0;
    for (int t = 0; t < threads; t++) {
        pthread_join(tid[t], NULL);
        acc += jobs[t].accepted;
    }
    free(tid);
    free(jobs);
    return (int64_t)acc;
}

/* Per-record verdicts (1 = accepted) on `threads` threads — the large-batch parity checker. */
struct vjob {
    struct job base;
    uint8_t* out;
};

static void* vworker(void* arg) {
    struct vjob* v = (struct vjob*)arg;
    struct job* j = &v->base;
    uint64_t maxlen = 0;
    for (uint64_t i = j->lo; i < j->hi; i++)
        if (j->off[i + 1] - j->off[i] > maxlen) maxlen = j->off[i + 1] - j->off[i];
    unsigned char* m = (unsigned char*)malloc(maxlen + 64);
    for (uint64_t i = j->lo; i < j->hi; i++) {
        const uint64_t len = j->off[i + 1] - j->off[i];
        int rc;
        if (j->fn) {
            unsigned long long mlen = 0;
            rc = j->fn(m, &mlen, j->blob + j->off[i], len, j->pk + 32 * i);
        } else {
            rc = oracle_sign_open(j->blob + j->off[i], len, j->pk + 32 * i);
        }
        v->out[i] = rc == 0;
    }
    free(m);
    return NULL;
}

int cpu_verdicts(const char* path, int use_sodium, const uint8_t* blob, const uint64_t* off, const uint8_t* pk,
                 uint64_t n, int threads, uint8_t* out) {
    open_fn fn = NULL;
    if (use_sodium) {
        void* h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
        if (!h) return -1;
        init_fn init = (init_fn)dlsym(h, "sodium_init");
        fn = (open_fn)dlsym(h, "crypto_sign_open");
        if (!init || !fn || init() < 0) return -1;
    }
    if (threads < 1) threads = 1;
    pthread_t* tid = (pthread_t*)calloc(threads, sizeof(pthread_t));
    struct vjob* jobs = (struct vjob*)calloc(threads, sizeof(struct vjob));
    for (int t = 0; t < threads; t++) {
        jobs[t].base.blob = blob;
        jobs[t].base.off = off;
        jobs[t].base.pk = pk;
        jobs[t].base.lo = n * t / threads;
        jobs[t].base.hi = n * (t + 1) / threads;
        jobs[t].base.fn = fn;
        jobs[t].out = out;
        pthread_create(&tid[t], NULL, vworker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) pthread_join(tid[t], NULL);
    free(tid);
    free(jobs);
    return 0;
}
