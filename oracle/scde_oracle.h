/* scde_oracle.h -- TEST INFRASTRUCTURE ONLY: shared declarations of the CPU
 * restatement (scde_oracle.c, bwpca_oracle.c). */
#ifndef SCDE_ORACLE_H
#define SCDE_ORACLE_H
#include <stdint.h>

/* glibc TYPE_3 rand() state (scde_oracle.c) */
typedef struct {
    int32_t tbl[31];
    int f, r;
} o_rng;

void o_srand(o_rng* g, unsigned int seed);
int o_rand(o_rng* g);

#endif
