// Fill kernels for strips of 64*2 rows (sa_fill.hip, one translation unit per R).
#define SA_FILL_R 2
#include "sa_fill.hip"
