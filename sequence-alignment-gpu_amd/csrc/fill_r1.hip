// Fill kernels for strips of 64*1 rows (sa_fill.hip, one translation unit per R).
#define SA_FILL_R 1
#include "sa_fill.hip"
