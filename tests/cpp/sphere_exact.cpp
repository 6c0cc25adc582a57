// TEST HARNESS: the exact f64 Sphere::hit (sphere.rs:77-96) the kernel's
// sphere rounds run (sphere_t_inv: correctly rounded divisions), compiled
// without contraction as the reference is.  Returns the accepted root or -1.
#include <cmath>

extern "C" double exact_sphere_t(const double c[3], double r, const double o[3], const double d[3], double tmin,
                                 double tmax) {
    const double oc[3] = {c[0] - o[0], c[1] - o[1], c[2] - o[2]};
    const double a = d[0] * d[0] + d[1] * d[1] + d[2] * d[2];
    const double h = d[0] * oc[0] + d[1] * oc[1] + d[2] * oc[2];
    const double cc = (oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2]) - r * r;
    const double disc = h * h - a * cc;
    if (disc < 0.0) return -1.0;
    const double sq = std::sqrt(disc);
    double root = (h - sq) / a;
    if (!(root >= tmin && root <= tmax)) {
        root = (h + sq) / a;
        if (!(root >= tmin && root <= tmax)) return -1.0;
    }
    return root;
}
