// genetic.cpp -- GeneticAlgorithm / GeneticAlgorithmMPI (GeneticAlgorithm.cpp:12-436,
// GeneticAlgorithmMPI.cpp:12-414) with each generation's population evaluated as one batch.
#include "GeneticAlgorithm.hpp"
#include "GeneticAlgorithmMPI.hpp"

#include <algorithm>
#include <cmath>
#include <ctime>
#include <iostream>
#include <stdexcept>

#include "../pnol_comm.hpp"
#include "../pnol_internal.hpp"
#include "device_util.hpp"

using namespace pnol;

// timeRand() of UtilityFunctionLibrary (absent): a uniform double in [0, 1) from splitmix64
double GARandom::next() {
    unsigned long long z = (state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    return (double)(z >> 11) * 0x1.0p-53;
}

// GeneticAlgorithm.cpp:312-340: a member equal to a later one is redrawn inside the box
void checkIndenticalChildAndReplace(vector<vector<double>>& Xpop, std::vector<double>& Xlb, std::vector<double>& Xub,
                                    vector<bool>& evaluateIndicator, GARandom& rng) {
    const int Npop = (int)Xpop.size();
    for (int i = 0; i < Npop; i++) {
        for (int k = i + 1; k < Npop; k++) {
            size_t same = 0;
            for (size_t j = 0; j < Xpop[i].size(); j++)
                if (Xpop[i][j] == Xpop[k][j]) same++;
            if (same == Xpop[i].size()) {
                for (size_t j = 0; j < Xpop[i].size(); j++) Xpop[i][j] = Xlb[j] + (Xub[j] - Xlb[j]) * rng.next();
                evaluateIndicator[i] = true;
            }
        }
    }
}

// GeneticAlgorithm.cpp:343-362: a coordinate outside the box is redrawn inside it
void checkPopulationBoundsAndReplace(vector<vector<double>>& Xpop, std::vector<double>& Xlb, std::vector<double>& Xub,
                                     vector<bool>& evaluateIndicator, GARandom& rng) {
    const int Npop = (int)Xpop.size();
    for (int i = 0; i < Npop; i++)
        for (size_t j = 0; j < Xlb.size(); j++)
            if (Xpop[i][j] > Xub[j] || Xpop[i][j] < Xlb[j]) {
                Xpop[i][j] = Xlb[j] + (Xub[j] - Xlb[j]) * rng.next();
                evaluateIndicator[i] = true;
            }
}

// GeneticAlgorithm.cpp:367-406 (selection sort by F): the first minimum among the members not
// yet placed -- the reference's order whenever its 2*max(F) sentinel exceeds every F
void popSort(vector<vector<double>>& Xpop, vector<double>& F) {
    const int Npop = (int)Xpop.size();
    vector<vector<double>> Xs(Npop);
    vector<double> Fs(Npop);
    vector<bool> taken(Npop, false);
    for (int k = 0; k < Npop; k++) {
        int best = -1;
        for (int i = 0; i < Npop; i++)
            if (!taken[i] && (best < 0 || F[i] < F[best])) best = i;
        taken[best] = true;
        Xs[k] = Xpop[best];
        Fs[k] = F[best];
    }
    Xpop.swap(Xs);
    F.swap(Fs);
}

namespace {

void print_row(const vector<double>& v) {
    for (double x : v) std::cout << x << " ";
    std::cout << std::endl;
}

// one batch of points through the objective: the device batch for device objectives (the
// objective's own per-point order), objEvalBatch otherwise
void eval_points(Objective* o, const vector<double>& Xs, int npts, int n, double* f) {
    if (npts <= 0) return;
    if (pnol_dobj* d = o->deviceObjective(n)) {
        check(pnol_dobj_eval_batch(d->ctx, d, Xs.data(), npts, f), "dobj_eval_batch(population)");
        o->countEvals(npts);
        return;
    }
    o->objEvalBatch(Xs.data(), npts, n, f);
}

// selection index of the crossover and mutation steps (GeneticAlgorithmMPI.cpp:134-146):
// round(u * Npop), clamped to the population (the reference reads one past it), accepted with
// probability fitness / maxFitness, never 0; uniform when no member past index 0 has positive
// fitness (every fitness 0, or all but the best tie with the worst -- a plateau objective --
// where the weighted draw would accept only u == 0 and never end)
int select_member(GARandom& rng, const vector<double>& fitness, double maxFitness, int Npop) {
    const bool flat = maxFitness == 0.0 ||
                      std::none_of(fitness.begin() + 1, fitness.begin() + Npop, [](double f) { return f > 0.0; });
    int index = 0;
    while (index == 0) {
        const int r = std::min((int)std::round(rng.next() * Npop), Npop - 1);
        const double u = rng.next();
        if (flat || u <= fitness[r] / maxFitness) index = r;
    }
    return index;
}

}  // namespace

void GeneticAlgorithm::evaluatePopulation(vector<vector<double>>& Xpop, vector<double>& F,
                                          vector<bool>& evaluateIndicator) {
    const int n = Xpop.empty() ? 0 : (int)Xpop[0].size();
    vector<int> who;
    vector<double> pts;
    for (int i = 0; i < Npop; i++)
        if (evaluateIndicator[i]) {
            who.push_back(i);
            pts.insert(pts.end(), Xpop[i].begin(), Xpop[i].end());
        }
    vector<double> f(who.size());
    eval_points(objPtr, pts, (int)who.size(), n, f.data());
    for (size_t k = 0; k < who.size(); k++) F[who[k]] = f[k];
}

void GeneticAlgorithm::evaluateGeneration(vector<vector<double>>& Xpop, vector<double>& F,
                                          vector<bool>& evaluateIndicator) {
    evaluatePopulation(Xpop, F, evaluateIndicator);
}

// GeneticAlgorithm.cpp:12-297 / GeneticAlgorithmMPI.cpp:12-278
void GeneticAlgorithm::runGA(std::vector<double>& X, std::vector<double>& Xlb, std::vector<double>& Xub, double& f0,
                             double& fOpt, bool root) {
    if (!objPtr) throw std::runtime_error("GeneticAlgorithm: no objective (setObjPtr)");
    if (Npop < 2) throw std::runtime_error("GeneticAlgorithm: Npop must be at least 2");
    const int Nparam = (int)X.size();
    if ((int)Xlb.size() != Nparam || (int)Xub.size() != Nparam) throw std::runtime_error("GeneticAlgorithm: bounds");
    vector<vector<double>> Xpop(Npop, vector<double>(Nparam)), XpopNew(Npop, vector<double>(Nparam));
    vector<double> F(Npop, 0), Fnew(Npop, 0), fitness(Npop, 0);
    vector<bool> evaluateIndicator(Npop, true);
    const int Nelite = (int)std::ceil(eliteFrac * Npop), NeliteMut = (int)std::ceil(eliteMutationFrac * Npop),
              Ncross = (int)std::ceil(crossFrac * Npop), Nrand = Npop - Nelite - NeliteMut - Ncross;
    if (Nrand <= 0)   // GeneticAlgorithmMPI.cpp:40-44 prints this and exits
        throw std::runtime_error("666 GA fractions set incorrectly. Sum must be less than 1 to avoid errors.");
    if (verbose && root) {
        std::cout << std::endl << "------------------------------------------------------------" << std::endl;
        std::cout << "Computing genetic algorithm with population " << std::endl;
        std::cout << "Nelite = " << Nelite << ", NeliteMut = " << NeliteMut << ", Ncross = " << Ncross
                  << ", Nrand = " << Nrand << std::endl;
        std::cout << "------------------------------------------------------------" << std::endl << std::endl;
    }
    GARandom rng{seeded ? seed : (unsigned long long)time(0)};
    for (int i = 0; i < Nparam; i++) Xpop[0][i] = X[i];
    for (int i = 1; i < Npop; i++)
        for (int j = 0; j < Nparam; j++) Xpop[i][j] = Xpop[0][j] + ((Xub[j] - Xlb[j]) * rng.next() + Xlb[j]);
    // the reference checks XpopNew (all zeros) here, which redraws all but its last member
    checkIndenticalChildAndReplace(XpopNew, Xlb, Xub, evaluateIndicator, rng);
    checkPopulationBoundsAndReplace(Xpop, Xlb, Xub, evaluateIndicator, rng);
    evaluateGeneration(Xpop, F, evaluateIndicator);
    f0 = F[0];
    popSort(Xpop, F);

    double FbestPrev = F[0];
    int Nstatic = 0, iter = 0;
    while (iter < maxGenerations) {
        if (verbose && root) {
            std::cout << "At generation = " << iter << " minimum of f = " << F[0] << "  at params:  ";
            print_row(Xpop[0]);
        }
        for (int k = 0; k < Npop; k++) fitness[k] = std::pow(F[Npop - 1] - F[k], 2);
        const double maxFitness = fitness[0];
        // 1. elite children
        for (int k = 0; k < Npop; k++) evaluateIndicator[k] = true;
        int popIdx = 0;
        for (int k = 0; k < Nelite; k++) {
            XpopNew[popIdx] = Xpop[popIdx];
            Fnew[popIdx] = F[popIdx];
            evaluateIndicator[popIdx] = false;
            popIdx++;
        }
        // 2. crossovers: every gene from a member chosen by fitness
        for (int k = 0; k < Ncross; k++) {
            vector<int> indices(Nparam, 0);
            for (int i = 0; i < Nparam; i++) indices[i] = select_member(rng, fitness, maxFitness, Npop);
            for (int i = 0; i < Nparam; i++) XpopNew[popIdx][i] = Xpop[indices[i]][i];
            popIdx++;
        }
        // 3. random mutations of a member chosen by fitness, the spread shrinking over generations
        const double spreadRatio = mutationSize * (maxGenerations - iter) / maxGenerations;
        for (int k = 0; k < Nrand; k++) {
            const int index = select_member(rng, fitness, maxFitness, Npop);
            for (int j = 0; j < Nparam; j++) {
                const double mutation = spreadRatio * (Xub[j] - Xlb[j]) * rng.next();
                XpopNew[popIdx][j] = Xpop[index][j] + mutation;
            }
            popIdx++;
        }
        // 4. mutations of the elite
        for (int k = 0; k < NeliteMut; k++) {
            for (int j = 0; j < Nparam; j++) {
                const int e = std::min((int)std::round(rng.next() * Nelite), Npop - 1);
                const double mutation = eliteMutationSize * (Xub[j] - Xlb[j]) * rng.next();
                XpopNew[popIdx][j] = Xpop[e][j] + mutation;
            }
            popIdx++;
        }
        // 5. repair, 6. evaluate, 7. sort
        checkIndenticalChildAndReplace(XpopNew, Xlb, Xub, evaluateIndicator, rng);
        checkPopulationBoundsAndReplace(XpopNew, Xlb, Xub, evaluateIndicator, rng);
        evaluateGeneration(XpopNew, Fnew, evaluateIndicator);
        popSort(XpopNew, Fnew);
        F = Fnew;
        Xpop = XpopNew;
        const double Fbest = F[0];
        Nstatic = (Fbest == FbestPrev) ? Nstatic + 1 : 0;
        if (Nstatic > NstaticGenerations) break;
        FbestPrev = Fbest;
        iter++;
    }
    generations = iter;
    fOpt = F[0];
    for (int i = 0; i < Nparam; i++) X[i] = Xpop[0][i];
    if (verbose && root) {
        std::cout << std::endl << "-----------------------------------------------------------------------------------"
                  << std::endl;
        std::cout << "Completed genetic algorithm." << std::endl;
        std::cout << "At generation = " << iter << " minimum of f = " << F[0] << "  at params:  ";
        print_row(Xpop[0]);
        std::cout << "-----------------------------------------------------------------------------------" << std::endl
                  << std::endl;
    }
}

void GeneticAlgorithm::findMinBnd(std::vector<double>& X, std::vector<double>& Xlb, std::vector<double>& Xub,
                                  double& f0, double& fOpt) {
    runGA(X, Xlb, Xub, f0, fOpt, true);
}

void GeneticAlgorithmMPI::findMinBnd(std::vector<double>& X, std::vector<double>& Xlb, std::vector<double>& Xub,
                                     double& f0, double& fOpt) {
    require_comm("GeneticAlgorithmMPI::findMinBnd");   // GeneticAlgorithmMPI.cpp:17-18
    runGA(X, Xlb, Xub, f0, fOpt, comm_rank() == 0);
}

// GeneticAlgorithmMPI.cpp:283-414.  Every rank takes the root's population (the reference
// zeroes the others' and sums), the members to evaluate go round-robin over the ranks, each rank
// evaluates its share as one batch, and every value is the owner's + 0.0 (the zero-padded sum).
void GeneticAlgorithmMPI::evaluatePopulationParallel(vector<vector<double>>& Xpop, vector<double>& F,
                                                     vector<bool>& evaluateIndicator) {
    const int P = comm_size(), me = comm_rank();
    const int n = Xpop.empty() ? 0 : (int)Xpop[0].size();
    pnol_ctx* hctx = nullptr;
    if (P > 1) {
        // the root's population, F and flags on every rank
        const size_t per = (size_t)Npop * n + 2 * (size_t)Npop;
        vector<double> mine(per), all(per * P);
        for (int i = 0; i < Npop; i++) {
            for (int j = 0; j < n; j++) mine[(size_t)i * n + j] = Xpop[i][j];
            mine[(size_t)Npop * n + i] = F[i];
            mine[(size_t)Npop * n + Npop + i] = evaluateIndicator[i] ? 1.0 : 0.0;
        }
        hctx = default_ctx_or_null();
        check(comm_allgather_host(hctx, mine.data(), all.data(), per), "allgather(population)");
        for (int i = 0; i < Npop; i++) {
            for (int j = 0; j < n; j++) Xpop[i][j] = all[(size_t)i * n + j] + 0.0;
            F[i] = all[(size_t)Npop * n + i] + 0.0;
            evaluateIndicator[i] = all[(size_t)Npop * n + Npop + i] != 0.0;
        }
    }
    // load balance (GeneticAlgorithmMPI.cpp:340-354): flagged members round-robin, others on the root
    vector<int> owner(Npop, 0);
    for (int i = 0, r = 0; i < Npop; i++)
        if (evaluateIndicator[i]) {
            owner[i] = r;
            r = (r + 1) % P;
        }
    vector<int> who;
    vector<double> pts;
    for (int i = 0; i < Npop; i++)
        if (evaluateIndicator[i] && owner[i] == me) {
            who.push_back(i);
            pts.insert(pts.end(), Xpop[i].begin(), Xpop[i].end());
        }
    vector<double> f(who.size());
    eval_points(objPtr, pts, (int)who.size(), n, f.data());
    if (P == 1) {
        for (size_t k = 0; k < who.size(); k++) F[who[k]] = f[k];
        return;
    }
    vector<double> mineF(Npop, 0.0), allF((size_t)Npop * P);
    for (int i = 0; i < Npop; i++) mineF[i] = F[i];   // the root's value stands for unflagged members
    for (size_t k = 0; k < who.size(); k++) mineF[who[k]] = f[k];
    check(comm_allgather_host(hctx, mineF.data(), allF.data(), Npop), "allgather(F)");
    for (int i = 0; i < Npop; i++) F[i] = allF[(size_t)owner[i] * Npop + i] + 0.0;
    for (int i = 0; i < Npop; i++)
        for (int j = 0; j < n; j++) Xpop[i][j] = Xpop[i][j] + 0.0;
}

void GeneticAlgorithmMPI::evaluateGeneration(vector<vector<double>>& Xpop, vector<double>& F,
                                             vector<bool>& evaluateIndicator) {
    evaluatePopulationParallel(Xpop, F, evaluateIndicator);
}
