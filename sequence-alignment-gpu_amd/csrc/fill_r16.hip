// Fill kernels for strips of 64*16 rows (sa_fill.hip, one translation unit per R).
#define SA_FILL_R 16
#include "sa_fill.hip"
