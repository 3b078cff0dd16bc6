/*
 * PNOL_Algorithm.hpp  (MI355X-native PNOL drop-in)
 *
 * Abstract optimizer bases, source compatible with Source/PNOL_Algorithm.hpp:22-65.
 * An algorithm holds a non-owning pointer to its objective (set with setObjPtr) and
 * overwrites X with the optimum.  The concrete classes (BFGS, BFGS_MPI, BFGS_Bnd, LevMarq,
 * LevMarqMPI) keep their dense state -- the inverse Hessian D, the Jacobian, J^T J -- in
 * HBM for the whole solve; only parameter-sized vectors cross PCIe.
 */
#ifndef PNOL_AMD_ALGORITHM_HPP_
#define PNOL_AMD_ALGORITHM_HPP_

#include <vector>

#include "PNOL_Objective.hpp"

// box-bounded scalar minimizer (BFGS_Bnd)
class AlgorithmBnd {
  protected:
    Objective* objPtr = nullptr;

  public:
    virtual ~AlgorithmBnd() {}
    virtual void findMinBnd(std::vector<double>& X, std::vector<double>& Xlb, std::vector<double>& Xub, double& f0,
                            double& fOpt) = 0;
    void setObjPtr(Objective& obj) { objPtr = &obj; }
};

// unconstrained scalar minimizer (BFGS, BFGS_MPI)
class Algorithm {
  protected:
    Objective* objPtr = nullptr;

  public:
    virtual ~Algorithm() {}
    virtual void findMin(std::vector<double>& X, double& f0, double& fOpt) = 0;
    void setObjPtr(Objective& obj) { objPtr = &obj; }
};

// least-squares minimizer over a residual vector (LevMarq, LevMarqMPI)
class MultiAlgorithm {
  protected:
    MultiObjective* mObjPtr = nullptr;

  public:
    virtual ~MultiAlgorithm() {}
    virtual void findMin(std::vector<double>& X, std::vector<double>& F0, std::vector<double>& F) = 0;
    void setObjPtr(MultiObjective& mObj) { mObjPtr = &mObj; }
};

#endif /* PNOL_AMD_ALGORITHM_HPP_ */
