/*
 * GeneticAlgorithmMPI.hpp  (MI355X-native PNOL drop-in)
 *
 * GeneticAlgorithm with the population evaluation dealt over the process communicator
 * (Source/GeneticAlgorithmMPI.hpp:32-82, GeneticAlgorithmMPI.cpp:283-414): the root's
 * population is what every rank evaluates (the reference zeroes the others and sums with
 * MPI_Allreduce), the members that need an evaluation go round-robin to the ranks, each rank
 * evaluates its share as one batch (on its GPU for device objectives), and the values are
 * assembled on every rank.  The reference's zero-padded sums turn -0.0 into +0.0 at P > 1; the
 * same + 0.0 is applied here, so results do not depend on how the values travel.
 */
#ifndef PNOL_AMD_GENETICALGORITHM_MPI_HPP_
#define PNOL_AMD_GENETICALGORITHM_MPI_HPP_

#include <vector>

#include "GeneticAlgorithm.hpp"

class GeneticAlgorithmMPI : public GeneticAlgorithm {
  protected:
    void evaluateGeneration(vector<vector<double>>& Xpop, vector<double>& F, vector<bool>& evaluateIndicator) override;

  public:
    void findMinBnd(std::vector<double>& X, std::vector<double>& Xlb, std::vector<double>& Xub, double& f0,
                    double& fOpt) override;

    // the reference's MPI signature (no graph flag)
    void setGAParams(int NpopIn, int maxGenerationsIn, double eliteFracIn, double crossFracIn,
                     double eliteMutationFracIn, double mutationSizeIn, double eliteMutationSizeIn,
                     double initialPopScalingIn, double NstaticGenerationsIn, bool verboseIn) {
        GeneticAlgorithm::setGAParams(NpopIn, maxGenerationsIn, eliteFracIn, crossFracIn, eliteMutationFracIn,
                                      mutationSizeIn, eliteMutationSizeIn, initialPopScalingIn, NstaticGenerationsIn,
                                      verboseIn, false);
    }

    void evaluatePopulationParallel(vector<vector<double>>& Xpop, vector<double>& F, vector<bool>& evaluateIndicator);

    GeneticAlgorithmMPI() {}
    ~GeneticAlgorithmMPI() override {}
};

#endif /* PNOL_AMD_GENETICALGORITHM_MPI_HPP_ */
