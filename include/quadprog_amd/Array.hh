// Array.hh — clean-room, layout-compatible subset of the reference's ArrayHH containers.
//
// The reference's solver boundary passes ArrayHH::Matrix<double> / ArrayHH::Vector<double>
// (reference include/QuadProgpp/QuadProg++.hh:69-72).  Their object layout is the ABI of the
// drop-in (reference include/QuadProgpp/Array.hh):
//   Vector<T> = { unsigned int n; T* v; }                           (Array.hh:57-59)
//   Matrix<T> = { unsigned int n; unsigned int m; T** v; }          (Array.hh:899-902)
//   Matrix storage: v[0] = new T[n*m] (row-major), v[i] = v[i-1] + m (Array.hh:910-919)
// This header reproduces exactly that layout and the members mgqp uses (sized constructors,
// resize, operator[], size/nrows/ncols, assignment, t()), so code compiled against either
// header links against libquadprog_amd.so.  Memory is owned with new[]/delete[] like the
// reference, so objects may cross between translation units built with either header.
#ifndef QUADPROG_AMD_ARRAY_HH
#define QUADPROG_AMD_ARRAY_HH

#include <stdexcept>

namespace ArrayHH {

template <typename T>
class Vector {
 public:
  Vector() : n(0), v(0) {}
  Vector(const unsigned int size) : n(size), v(new T[size]) {}
  Vector(const T& a, const unsigned int size) : n(size), v(new T[size]) {
    for (unsigned int i = 0; i < n; i++) v[i] = a;
  }
  Vector(const T* a, const unsigned int size) : n(size), v(new T[size]) {
    for (unsigned int i = 0; i < n; i++) v[i] = a[i];
  }
  Vector(const Vector& o) : n(o.n), v(new T[o.n]) {
    for (unsigned int i = 0; i < n; i++) v[i] = o.v[i];
  }
  ~Vector() { delete[] v; }

  inline T& operator[](const unsigned int& i) { return v[i]; }
  inline const T& operator[](const unsigned int& i) const { return v[i]; }
  inline unsigned int size() const { return n; }

  inline void resize(const unsigned int size) {
    if (size == n) return;  // same size: contents kept (reference semantics)
    delete[] v;
    v = new T[size];
    n = size;
  }
  inline void resize(const T& a, const unsigned int size) {
    resize(size);
    for (unsigned int i = 0; i < n; i++) v[i] = a;
  }
  Vector& operator=(const Vector& o) {
    if (this != &o) {
      resize(o.n);
      for (unsigned int i = 0; i < n; i++) v[i] = o.v[i];
    }
    return *this;
  }
  Vector& operator=(const T& a) {
    for (unsigned int i = 0; i < n; i++) v[i] = a;
    return *this;
  }

 private:
  unsigned int n;
  T* v;
};

template <typename T>
class Matrix {
 public:
  Matrix() : n(0), m(0), v(0) {}
  Matrix(const unsigned int rows, const unsigned int cols) : n(rows), m(cols), v(0) { alloc(); }
  Matrix(const T& a, const unsigned int rows, const unsigned int cols) : n(rows), m(cols), v(0) {
    alloc();
    for (unsigned int i = 0; i < n; i++)
      for (unsigned int j = 0; j < m; j++) v[i][j] = a;
  }
  Matrix(const T* a, const unsigned int rows, const unsigned int cols) : n(rows), m(cols), v(0) {
    alloc();
    for (unsigned int i = 0; i < n; i++)
      for (unsigned int j = 0; j < m; j++) v[i][j] = *a++;
  }
  Matrix(const Matrix& o) : n(o.n), m(o.m), v(0) {
    alloc();
    for (unsigned int i = 0; i < n; i++)
      for (unsigned int j = 0; j < m; j++) v[i][j] = o.v[i][j];
  }
  ~Matrix() { release(); }

  inline T* operator[](const unsigned int& i) { return v[i]; }
  inline const T* operator[](const unsigned int& i) const { return v[i]; }
  inline unsigned int nrows() const { return n; }
  inline unsigned int ncols() const { return m; }

  inline void resize(const unsigned int rows, const unsigned int cols) {
    if (rows == n && cols == m) return;
    release();
    n = rows;
    m = cols;
    alloc();
  }
  inline void resize(const T& a, const unsigned int rows, const unsigned int cols) {
    resize(rows, cols);
    for (unsigned int i = 0; i < n; i++)
      for (unsigned int j = 0; j < m; j++) v[i][j] = a;
  }
  Matrix& operator=(const Matrix& o) {
    if (this != &o) {
      resize(o.n, o.m);
      for (unsigned int i = 0; i < n; i++)
        for (unsigned int j = 0; j < m; j++) v[i][j] = o.v[i][j];
    }
    return *this;
  }
  Matrix& operator=(const T& a) {
    for (unsigned int i = 0; i < n; i++)
      for (unsigned int j = 0; j < m; j++) v[i][j] = a;
    return *this;
  }

 private:
  // Row-pointer table + one contiguous row-major block.  Unlike the reference (Array.hh:1060,
  // which writes v[0] into a zero-length table when n == 0), a 0-row matrix gets a 1-entry
  // table so the block pointer always has a home.
  void alloc() {
    v = new T*[n > 0 ? n : 1];
    v[0] = new T[(size_t)n * m];
    for (unsigned int i = 1; i < n; i++) v[i] = v[i - 1] + m;
  }
  void release() {
    if (v) {
      delete[] v[0];
      delete[] v;
      v = 0;
    }
  }
  unsigned int n;
  unsigned int m;
  T** v;
};

// Transposed copy (reference Array.hh:2463-2472), used by mgqp to pass CE^T / CI^T.
template <typename T>
Matrix<T> t(const Matrix<T>& a) {
  Matrix<T> r(a.ncols(), a.nrows());
  for (unsigned int i = 0; i < a.nrows(); i++)
    for (unsigned int j = 0; j < a.ncols(); j++) r[j][i] = a[i][j];
  return r;
}

}  // namespace ArrayHH

#endif  // QUADPROG_AMD_ARRAY_HH
