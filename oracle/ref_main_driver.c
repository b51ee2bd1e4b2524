/* oracle/ref_main_driver.c -- TEST INFRASTRUCTURE.
 * Runs the reference program's own main() (PQP_CPU.c:935-1040, compiled
 * unmodified into _ref/libpqp_ref.so with main renamed pqp_ref_main) with
 * libpqp.so placed FIRST in the symbol search order, so every call main()
 * makes to input/Gauss_Jordan/computeFp/computeMp/convertToDual/
 * solveQuadraticDual/computeUfromY/computeCost resolves to the GPU drop-ins of
 * include/pqp.h -- the reference's driver running on the new library. */
int pqp_ref_main(void);
int main(void) { return pqp_ref_main(); }
