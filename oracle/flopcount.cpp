/*
 * flopcount.cpp -- TEST INFRASTRUCTURE (oracle). Never linked into the product.
 * The counter of the op-counting build (flopcount.hpp) and its reader.
 */
thread_local long long orc_flop_counter = 0;

extern "C" long long orc_flops_take(void)
{
    const long long n = orc_flop_counter;
    orc_flop_counter = 0;
    return n;
}
