/* crashline.c -- bench.py insurance: if a process dies on a fatal signal (a GPU fault makes the
 * HSA runtime call abort(); a bad pointer gives SIGSEGV / SIGBUS) after the headline was
 * measured, or is terminated (SIGTERM: a launcher's time limit, torchrun passing one on), write
 * the last armed JSON line to the given fd before dying, so the one-line contract still holds.
 * Only async-signal-safe calls (write, signal, raise) in the handler.
 *
 *   crashline_arm(fd, line)  copy `line` (+ '\n') into a static buffer; install the handlers
 *   crashline_disarm()       forget the line (the normal emit path printed it)
 */
#include <signal.h>
#include <string.h>
#include <unistd.h>

static char g_line[1 << 16];
static volatile sig_atomic_t g_len = 0;
static volatile sig_atomic_t g_fd = -1;

static void on_fatal(int sig) {
  int len = g_len, fd = g_fd;
  g_len = 0;
  if (len > 0 && fd >= 0) {
    const char* p = g_line;
    while (len > 0) {
      ssize_t k = write(fd, p, (size_t)len);
      if (k <= 0) break;
      p += k;
      len -= (int)k;
    }
  }
  signal(sig, SIG_DFL);
  raise(sig);
}

int crashline_arm(int fd, const char* line) {
  size_t n = strlen(line);
  if (n + 2 > sizeof g_line) return -1;
  g_len = 0;  /* never expose a half-copied line */
  memcpy(g_line, line, n);
  g_line[n] = '\n';
  g_fd = fd;
  g_len = (sig_atomic_t)(n + 1);
  {  /* (re)installed on every arm: a library loaded since may have replaced it */
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_handler = on_fatal;
    sigemptyset(&sa.sa_mask);
    sa.sa_flags = SA_RESETHAND;
    sigaction(SIGABRT, &sa, NULL);
    sigaction(SIGSEGV, &sa, NULL);
    sigaction(SIGBUS, &sa, NULL);
    sigaction(SIGFPE, &sa, NULL);
    sigaction(SIGILL, &sa, NULL);
    sigaction(SIGTERM, &sa, NULL);
  }
  return 0;
}

void crashline_disarm(void) { g_len = 0; }
