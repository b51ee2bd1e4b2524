// pqp_cli -- the reference program (PQP_CPU.c main, :935-1040) on the GPU:
// reads <dir>/{Qp_inv,Fp1,...}.txt (default ./example, as the reference does),
// runs setup, the solve and the recovery on the MI355X and prints the
// reference's stdout byte for byte.
#include <cstdio>

#include "../../include/pqp.h"

int main(int argc, char** argv) {
    const char* dir = argc > 1 ? argv[1] : "./example";
    const int rc = pqp_run_example(dir, nullptr);
    if (rc != PQP_OK) {
        std::fprintf(stderr, "pqp_cli: %s\n", pqp_last_error());
        return 1;
    }
    return 0;
}
