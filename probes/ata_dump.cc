// Diagnostics (not product, not tests): the CPU oracle with a hook that
// records every packed A^T A the LO estimators hand to ata_null_vector.
#include <vector>
namespace scm { namespace geom { void ata_hook(const double* a); } }
#define SCM_GEOM_ATA_HOOK ata_hook
#include "../oracle/oracle.cc"
static std::vector<double> g_ata;
void scm::geom::ata_hook(const double* a) { g_ata.insert(g_ata.end(), a, a + 45); }
extern "C" long ata_dump_count() { return (long)(g_ata.size() / 45); }
extern "C" void ata_dump_get(double* out) { std::copy(g_ata.begin(), g_ata.end(), out); g_ata.clear(); }
