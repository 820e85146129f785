// Developer aid: SFHE_CRASH_TRACE=1 installs a SIGSEGV/SIGABRT handler that
// writes the native backtrace (raw addresses + the library's load address from
// /proc/self/maps, for addr2line) to stderr before the process dies.
#include <execinfo.h>
#include <fcntl.h>
#include <signal.h>
#include <unistd.h>

#include <cstdlib>
#include <cstring>

namespace {

void writeStr(const char* s) { (void)!write(2, s, std::strlen(s)); }

void handler(int sig) {
    writeStr(sig == SIGSEGV ? "\n[sfhe] SIGSEGV, backtrace:\n" : "\n[sfhe] fatal signal, backtrace:\n");
    void* frames[64];
    const int n = backtrace(frames, 64);
    backtrace_symbols_fd(frames, n, 2);
    writeStr("[sfhe] mappings of libsfhe:\n");
    const int fd = open("/proc/self/maps", O_RDONLY);
    if (fd >= 0) {
        char buf[8192];
        ssize_t r;
        // print only lines naming the library (line-buffered scan)
        char line[512];
        size_t len = 0;
        while ((r = read(fd, buf, sizeof buf)) > 0) {
            for (ssize_t i = 0; i < r; ++i) {
                if (len < sizeof line - 1) line[len++] = buf[i];
                if (buf[i] == '\n') {
                    line[len] = 0;
                    if (std::strstr(line, "libsfhe")) writeStr(line);
                    len = 0;
                }
            }
        }
        close(fd);
    }
    signal(sig, SIG_DFL);
    raise(sig);
}

struct Install {
    Install() {
        const char* v = std::getenv("SFHE_CRASH_TRACE");
        if (!v || *v == '0') return;
        signal(SIGSEGV, handler);
        signal(SIGABRT, handler);
    }
} install;

}  // namespace
