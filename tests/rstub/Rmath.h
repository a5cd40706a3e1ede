/* TEST INFRASTRUCTURE: see Rinternals.h */
double unif_rand(void);
