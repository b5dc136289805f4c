// Fill kernels for strips of 64*8 rows (sa_fill.hip, one translation unit per R).
#define SA_FILL_R 8
#include "sa_fill.hip"
