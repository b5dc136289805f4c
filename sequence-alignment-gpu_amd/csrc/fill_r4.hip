// Fill kernels for strips of 64*4 rows (sa_fill.hip, one translation unit per R).
#define SA_FILL_R 4
#include "sa_fill.hip"
