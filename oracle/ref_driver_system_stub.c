/* TEST INFRASTRUCTURE ONLY — linked into the reference's own experiment
 * drivers built by `make -C oracle drivers` (never into the product).
 *
 * experiments/src/vertex-classification.cpp:152-158,170-195 shells out to
 * yskip (an un-vendored external skip-gram trainer), a Perl converter and a
 * Python classifier after writing each corpus — the downstream embedding step,
 * outside the walk path.  The driver is linked with
 * -Wl,--wrap=system so those calls land here: the command is logged and
 * reported as successful, and the driver's own code runs unchanged. */
#include <stdio.h>

int __wrap_system(const char* command)
{
    fprintf(stderr, "[downstream step not run] %s\n", command ? command : "(null)");
    return 0;
}
