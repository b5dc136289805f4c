// Fill kernels for R = 1 chains of alphabets larger than 4 that read copy 0 of their text profiles
// (kArr8A, sa_fill.h): a code object of its own, so the DNA kernels of fill_r1.hip are unchanged.
#define SA_FILL_R 1
#define SA_FILL_ALIGN 1
#include "sa_fill.hip"
