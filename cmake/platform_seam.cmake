# ctest `platform_seam`: Linux-only system interfaces appear in src/ only under
# src/platform/linux*.cc (the default build's platform layer) and src/helper/ (the in-container
# agent, Linux by design). Everything else compiles against POSIX (-DDEVSPACE_PORTABLE=ON).
# Same rule as tests/test_platform.py::test_linux_only_calls_stay_behind_the_platform_layer.
file(GLOB_RECURSE SRCS ${ROOT}/src/*.cc ${ROOT}/src/*.h)
set(PATTERNS "inotify_" "epoll_" "prctl\\(" "pipe2\\(" "accept4\\(" "eventfd\\(" "MSG_NOSIGNAL" "SOCK_CLOEXEC"
             "O_TMPFILE" "/proc/self" "sys/inotify\\.h" "sys/epoll\\.h" "sys/prctl\\.h" "sys/eventfd\\.h" "signalfd"
             "timerfd"
             # Linux or glibc only (macOS's headers lack them)
             "F_SETPIPE_SZ" "TCP_QUICKACK" "TCP_USER_TIMEOUT" "TCP_KEEPIDLE" "SO_PEERCRED" "splice\\(" "memfd_create"
             "getrandom\\(" "CLOCK_BOOTTIME" "posix_fadvise" "fallocate\\(" "statx\\(" "SOCK_NONBLOCK" "renameat2"
             "copy_file_range" "MSG_MORE" "<endian\\.h>" "<byteswap\\.h>" "<malloc\\.h>" "<sys/sendfile\\.h>"
             "<linux/" "be64toh" "htobe64" "be32toh" "htobe32" "strchrnul" "memrchr" "get_nprocs" "sys/sysinfo\\.h"
             "program_invocation_name" "pthread_tryjoin_np" "ppoll\\(")
set(BAD "")
foreach(f ${SRCS})
  if(f MATCHES "/src/platform/linux[^/]*$" OR f MATCHES "/src/helper/")
    continue()
  endif()
  file(STRINGS ${f} LINES ENCODING UTF-8)
  foreach(l ${LINES})
    if(l MATCHES "^[ \t]*//")  # documentation of the seam itself
      continue()
    endif()
    foreach(p ${PATTERNS})
      if(l MATCHES "${p}")
        list(APPEND BAD "${f}: ${l}")
      endif()
    endforeach()
  endforeach()
endforeach()
if(BAD)
  list(JOIN BAD "\n" MSG)
  message(FATAL_ERROR "Linux-only calls outside src/platform/linux*:\n${MSG}")
endif()
