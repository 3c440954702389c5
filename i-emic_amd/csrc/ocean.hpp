/*
 * ocean.hpp -- header-only C++ host class over the C ABI (include/iemic.h), with the
 * method names and argument meaning of the reference's Ocean model
 * (src/ocean/Ocean.H; the calls Continuation and transient/Newton make)
 * and an Epetra-shaped vector (Update / Scale / PutScalar / Norm2 / Dot / GlobalLength).
 *
 *   reference                                  here
 *   Ocean::computeRHS()            Ocean.C:1267    computeRHS()      -> iemic_rhs
 *   Ocean::computeJacobian()       Ocean.C:1287    computeJacobian() -> iemic_jacobian
 *   Ocean::solve(rhs)              Ocean.C:1060    solve(rhs)        -> iemic_prec_compute + iemic_solve
 *   Ocean::applyMatrix(in, out)    Ocean.C:1352    applyMatrix       -> iemic_spmv
 *   Ocean::getState/getSolution/getRHS('C'|'V')    Ocean.C:1302-1318
 *   Ocean::setPar/getPar(std::string, double)      THCM::par2int names (THCM.C:1754-1807)
 *   Ocean::preProcess / postProcess                Ocean.C:790-801
 *
 * Errors throw std::runtime_error carrying iemic_last_error() (the reference throws via
 * its ERROR macro).  No CPU fallback exists: construction throws without a GPU.
 */
#ifndef IEMIC_OCEAN_HPP
#define IEMIC_OCEAN_HPP

#include <cmath>
#include <map>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/iemic.h"

namespace iemic {

inline void check(int rc, const char* what)
{
    if (rc != 0)
        throw std::runtime_error(std::string(what) + " failed (rc=" + std::to_string(rc) +
                                 "): " + iemic_last_error());
}

/* Epetra_Vector-shaped host vector in the reference's global row order. */
class Vector {
  public:
    explicit Vector(size_t n = 0, double v = 0.0) : v_(n, v) {}
    size_t GlobalLength() const { return v_.size(); }
    double* data() { return v_.data(); }
    const double* data() const { return v_.data(); }
    double& operator[](size_t i) { return v_[i]; }
    double operator[](size_t i) const { return v_[i]; }
    void PutScalar(double a) { std::fill(v_.begin(), v_.end(), a); }
    void Scale(double a) { for (double& x : v_) x *= a; }
    /* this = a*X + b*this  (Epetra_MultiVector::Update) */
    void Update(double a, const Vector& X, double b)
    {
        for (size_t i = 0; i < v_.size(); i++) v_[i] = a * X.v_[i] + b * v_[i];
    }
    double Dot(const Vector& X) const
    {
        double s = 0.0;
        for (size_t i = 0; i < v_.size(); i++) s += v_[i] * X.v_[i];
        return s;
    }
    double Norm2() const { return std::sqrt(Dot(*this)); }

  private:
    std::vector<double> v_;
};

class Ocean {
  public:
    /* grid: the THCM ParameterList subset; landm: (n+2)(m+2)(l+2) global mask */
    Ocean(const iemic_grid& grid, const std::vector<int>& landm)
    {
        if (iemic_abi_version() != IEMIC_ABI_VERSION)
            throw std::runtime_error("libiemic_amd was built from another iemic.h (ABI version " +
                                     std::to_string(iemic_abi_version()) + ", header " +
                                     std::to_string(IEMIC_ABI_VERSION) + ")");
        check(iemic_create(&ctx_, &grid, landm.data()), "iemic_create");
        N_ = (size_t)iemic_nrows(ctx_);
        state_ = std::make_shared<Vector>(N_);
        rhs_ = std::make_shared<Vector>(N_);
        sol_ = std::make_shared<Vector>(N_);
        /* Belos defaults of Ocean::getDefaultInitParameters (Ocean.C:2232-2237) */
        krylov_ = iemic_krylov{1e-8, 500, 0, 2, 12, 0, 4, /*method FGMRES*/ 0, 1, 1, 0.95, 0, 4, 0.7, 0, 0, /*Schur passes*/ 2};
    }
    ~Ocean() { iemic_destroy(ctx_); }
    Ocean(const Ocean&) = delete;
    Ocean& operator=(const Ocean&) = delete;

    /* ---- Model interface -------------------------------------------------------- */
    void computeRHS() { check(iemic_rhs(ctx_, rhs_->data()), "computeRHS"); }
    void computeJacobian() { check(iemic_jacobian(ctx_), "computeJacobian"); }
    void applyMatrix(const Vector& in, Vector& out)
    {
        check(iemic_spmv(ctx_, in.data(), out.data()), "applyMatrix");
    }
    void buildPreconditioner(bool force = false)
    {
        if (recompPrec_ || force) {
            check(iemic_prec_compute(ctx_, &krylov_), "buildPreconditioner");
            recompPrec_ = false;
        }
    }
    void applyPrecon(const Vector& in, Vector& out)
    {
        check(iemic_prec_apply(ctx_, in.data(), out.data()), "applyPrecon");
    }
    /* J sol = rhs (Ocean::solve); the solution is in getSolution() */
    void solve(const Vector& rhs)
    {
        buildPreconditioner();
        check(iemic_solve(ctx_, rhs.data(), sol_->data(), &krylov_, &lastSolve_), "solve");
    }
    void preProcess() { recompPrec_ = true; }
    void postProcess() {}

    /* ---- state (mode 'C' = copy, 'V' = view of the host mirror) ----------------- */
    void setState(const Vector& x)
    {
        *state_ = x;
        check(iemic_set_state(ctx_, x.data()), "setState");
    }
    std::shared_ptr<Vector> getState(char mode)
    {
        check(iemic_get_state(ctx_, state_->data()), "getState");
        return mode == 'V' ? state_ : std::make_shared<Vector>(*state_);
    }
    std::shared_ptr<Vector> getRHS(char mode)
    {
        return mode == 'V' ? rhs_ : std::make_shared<Vector>(*rhs_);
    }
    std::shared_ptr<Vector> getSolution(char mode)
    {
        return mode == 'V' ? sol_ : std::make_shared<Vector>(*sol_);
    }

    /* ---- parameters (THCM::par2int names) ---------------------------------------- */
    void setPar(const std::string& name, double v) { check(iemic_set_par(ctx_, parIndex(name), v), "setPar"); }
    double getPar(const std::string& name)
    {
        double v = 0.0;
        check(iemic_get_par(ctx_, parIndex(name), &v), "getPar");
        return v;
    }
    static int parIndex(const std::string& name)
    {
        static const std::map<std::string, int> idx = {
            {"AL_T", 1}, {"Rayleigh-Number", 2}, {"Vertical Ekman-Number", 3},
            {"Horizontal Ekman-Number", 4}, {"Rossby-Number", 5}, {"MIXP", 6}, {"RESC", 7},
            {"SPL1", 8}, {"Salinity Homotopy", 9}, {"Solar Forcing", 10},
            {"Horizontal Peclet-Number", 11}, {"Vertical Peclet-Number", 12}, {"P_VC", 13},
            {"LAMB", 14}, {"Salinity Forcing", 15}, {"Wind Forcing", 16},
            {"Temperature Forcing", 17}, {"Nonlinear Factor", 18}, {"Combined Forcing", 19},
            {"ARCL", 20}, {"NLES", 21}, {"IFRICB", 22}, {"CONT", 23}, {"Energy", 24},
            {"ALPC", 25}, {"CMPR", 26}, {"Flux Perturbation", 27},
            {"Salinity Perturbation", 28}, {"MKAP", 29}, {"SPL2", 30}};
        auto it = idx.find(name);
        if (it == idx.end()) throw std::runtime_error("invalid THCM parameter: " + name);
        return it->second;
    }

    /* ---- Belos settings (names of Ocean's solver ParameterList) ----------------- */
    iemic_krylov& solverParameters() { return krylov_; }
    const iemic_solve_info& lastSolve() const { return lastSolve_; }

    /* device-resident Newton step (transient/Newton.H:92-99 shape).  The update is applied
     * even when the linear solve missed its tolerance (IEMIC_ENOCONV, a warning), as the
     * reference's Newton / Continuation go on with the unconverged correction unless
     * rejectFailedNewton is set: the caller reads info.solve.converged.  Errors throw. */
    iemic_newton_info newtonStep()
    {
        iemic_newton_info info{};
        const int rc = iemic_newton_step(ctx_, &krylov_, &info);
        if (rc != IEMIC_ENOCONV) check(rc, "newtonStep");
        return info;
    }

    size_t nrows() const { return N_; }
    iemic_ctx* handle() { return ctx_; }

  private:
    iemic_ctx* ctx_ = nullptr;
    size_t N_ = 0;
    std::shared_ptr<Vector> state_, rhs_, sol_;
    iemic_krylov krylov_{};
    iemic_solve_info lastSolve_{};
    bool recompPrec_ = true;
};

}  // namespace iemic
#endif
