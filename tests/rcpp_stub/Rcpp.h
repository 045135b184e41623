// Test-only declarations of the Rcpp / R API subset that
// multiview-clustering_amd/R/multiview_gibbs.cpp uses, so that file can be
// compile-checked here (R and Rcpp are absent from this image).  Not an Rcpp
// implementation: nothing links against it.  Signatures follow Rcpp 1.0's
// public API (Rcpp/vector/Vector.h, Rcpp/Named.h, Rcpp/exceptions.h).
#pragma once
#include <cstddef>
#include <string>

typedef struct SEXPREC *SEXP;
extern "C" int Rf_isMatrix(SEXP);

namespace R {
double unif_rand();
}

namespace Rcpp {
[[noreturn]] void stop(const std::string &message);

template <int RTYPE>
class Vector {
 public:
  Vector();
  explicit Vector(SEXP x);
  explicit Vector(int n);
  template <class It>
  Vector(It first, It last);
  int size() const;
  double *begin();
  double *end();
  operator SEXP() const;
  struct Proxy {
    operator SEXP() const;
    template <class T>
    Proxy &operator=(const T &);
  };
  Proxy operator[](int i);
  Proxy operator[](int i) const;
  template <class... T>
  static Vector create(const T &...);
};
typedef Vector<14> NumericVector;
typedef Vector<13> IntegerVector;
typedef Vector<19> List;

class NumericMatrix {
 public:
  explicit NumericMatrix(SEXP x);
  int nrow() const;
  int ncol() const;
  double operator()(int i, int j) const;
};

struct NamedArg {
  template <class T>
  NamedArg &operator=(const T &);
};
NamedArg Named(const std::string &name);
}  // namespace Rcpp
