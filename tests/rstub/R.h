/* TEST INFRASTRUCTURE: see Rinternals.h */
#include "Rinternals.h"
