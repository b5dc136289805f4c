// Fill kernels for strips of 64*16 rows (see sa_engine.hip: one translation unit per R).
#define SA_FILL_R 16
#include "sa_engine.hip"
