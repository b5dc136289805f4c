// Fill kernels for strips of 64*32 rows (sa_fill.hip, one translation unit per R).
#define SA_FILL_R 32
#include "sa_fill.hip"
