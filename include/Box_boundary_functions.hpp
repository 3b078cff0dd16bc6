/*
 * Box_boundary_functions.hpp  (MI355X-native PNOL drop-in)
 *
 * Box helpers used by the bounded BFGS (Source/Box_boundary_functions.hpp and
 * BFGS_with_bnd_linsearch_MPI.cpp:665-708).
 */
#ifndef PNOL_AMD_BOX_BOUNDARY_FUNCTIONS_HPP_
#define PNOL_AMD_BOX_BOUNDARY_FUNCTIONS_HPP_

#include <vector>

// An X_i more than |bound|/1000 outside [Xlb_i, Xub_i] is replaced by the box midpoint
// (Box_boundary_functions.cpp:11-40); the warning prints on rank 0.
void checkBoxBounds(std::vector<double>& X, std::vector<double>& Xlb, std::vector<double>& Xub);

// Largest step along p that stays in the box: min over i of the first positive crossing
// (Xub - X)/p or (Xlb - X)/p, 0 where neither is positive (BFGS_with_bnd_linsearch_MPI.cpp:665-708).
double computeAlphaBnd(std::vector<double>& X, std::vector<double>& Xlb, std::vector<double>& Xub,
                       std::vector<double>& p);

#endif /* PNOL_AMD_BOX_BOUNDARY_FUNCTIONS_HPP_ */
