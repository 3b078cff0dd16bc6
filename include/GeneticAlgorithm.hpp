/*
 * GeneticAlgorithm.hpp  (MI355X-native PNOL drop-in)
 *
 * The reference's box-bounded genetic algorithm (Source/GeneticAlgorithm.hpp:37-87,
 * GeneticAlgorithm.cpp:12-300): elite children, fitness-weighted crossovers, spread-shrinking
 * random mutations, mutations of the elite, identical-child and bound repair, population sort.
 * The population of a generation is evaluated as ONE batch: on the device when the objective
 * provides deviceObjective() (pnol_dobj_eval_batch, each point in the objective's own order),
 * otherwise through Objective::objEvalBatch.
 *
 * Differences from the reference, all documented in DESIGN.md (row f4):
 *  - timeRand() (UtilityFunctionLibrary, absent) is a uniform double from a per-solver
 *    splitmix64 stream, seeded with time(0) like the reference's srand, or with setSeed();
 *  - a selection draw round(u * Npop) that lands on Npop (the reference then reads fitness[Npop],
 *    one past the end) is clamped to Npop - 1;
 *  - when every member has the same F (max fitness 0) the reference's selection loop never
 *    ends (0/0 comparisons); here selection is uniform in that case;
 *  - popSort takes the first minimum among the members not yet placed, which is the
 *    reference's order whenever max F > 0 (its 2*FMax sentinel breaks otherwise);
 *  - graph (VTK rendering) is accepted and ignored: plotting is out of scope.
 */
#ifndef PNOL_AMD_GENETICALGORITHM_HPP_
#define PNOL_AMD_GENETICALGORITHM_HPP_

#include <vector>

#include "PNOL_Algorithm.hpp"

using namespace std;

// the reference's free helpers (GeneticAlgorithm.hpp:30-32); `rng` is the solver's stream
struct GARandom {
    unsigned long long state;
    double next();   // uniform in [0, 1)
};
void checkPopulationBoundsAndReplace(vector<vector<double>>& Xpop, std::vector<double>& Xlb, std::vector<double>& Xub,
                                     vector<bool>& evaluateIndicator, GARandom& rng);
void checkIndenticalChildAndReplace(vector<vector<double>>& Xpop, std::vector<double>& Xlb, std::vector<double>& Xub,
                                    vector<bool>& evaluateIndicator, GARandom& rng);
void popSort(vector<vector<double>>& Xpop, vector<double>& F);

class GeneticAlgorithm : public AlgorithmBnd {
  protected:
    int Npop;
    int maxGenerations;
    double eliteFrac, crossFrac, eliteMutationFrac;
    double mutationSize, eliteMutationSize;
    double initialPopScaling;
    double NstaticGenerations;
    bool verbose;
    bool graph;
    bool seeded = false;
    unsigned long long seed = 0;
    int generations = 0;
    // the population evaluation of one generation (GeneticAlgorithm.cpp:301-310); the MPI class
    // deals it over the ranks
    virtual void evaluateGeneration(vector<vector<double>>& Xpop, vector<double>& F, vector<bool>& evaluateIndicator);
    void runGA(std::vector<double>& X, std::vector<double>& Xlb, std::vector<double>& Xub, double& f0, double& fOpt,
               bool root);

  public:
    void findMinBnd(std::vector<double>& X, std::vector<double>& Xlb, std::vector<double>& Xub, double& f0,
                    double& fOpt) override;

    void setGAParams(int NpopIn, int maxGenerationsIn, double eliteFracIn, double crossFracIn,
                     double eliteMutationFracIn, double mutationSizeIn, double eliteMutationSizeIn,
                     double initialPopScalingIn, double NstaticGenerationsIn, bool verboseIn, bool graphIn) {
        Npop = NpopIn; eliteFrac = eliteFracIn; crossFrac = crossFracIn; eliteMutationFrac = eliteMutationFracIn;
        maxGenerations = maxGenerationsIn; mutationSize = mutationSizeIn; eliteMutationSize = eliteMutationSizeIn;
        NstaticGenerations = NstaticGenerationsIn; verbose = verboseIn; initialPopScaling = initialPopScalingIn;
        graph = graphIn;
    }

    void evaluatePopulation(vector<vector<double>>& Xpop, vector<double>& F, vector<bool>& evaluateIndicator);

    // extensions: a reproducible stream (default: time(0), as the reference's srand), and the
    // number of generations the last findMinBnd ran
    void setSeed(unsigned long long s) { seed = s; seeded = true; }
    int getGenerations() const { return generations; }

    GeneticAlgorithm()
        : Npop(100), maxGenerations(1000), eliteFrac(0.1), crossFrac(0.3), eliteMutationFrac(0.2), mutationSize(0.5),
          eliteMutationSize(0.01), initialPopScaling(0.5), NstaticGenerations(50), verbose(false), graph(false) {}
    ~GeneticAlgorithm() override {}
};

#endif /* PNOL_AMD_GENETICALGORITHM_HPP_ */
