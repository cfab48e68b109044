/*
 * shim_log.h -- minimal stand-in for Shadow's logger macros (support/logger/logger.h:19-28)
 * so the shim keeps the reference's messages and levels.  Inside Shadow a maintainer maps
 * these onto error()/critical()/warning()/message()/info()/debug().
 */
#ifndef SHADOWTOPO_SHIM_LOG_H
#define SHADOWTOPO_SHIM_LOG_H

enum { ST_ERROR = 0, ST_CRITICAL = 1, ST_WARNING = 2, ST_MESSAGE = 3, ST_INFO = 4, ST_DEBUG = 5 };

void shadowtopo_log(int level, const char* func, const char* fmt, ...) __attribute__((format(printf, 3, 4)));
int shadowtopo_log_enabled(int level);

#define st_error(...) shadowtopo_log(ST_ERROR, __func__, __VA_ARGS__)
#define st_critical(...) shadowtopo_log(ST_CRITICAL, __func__, __VA_ARGS__)
#define st_warning(...) shadowtopo_log(ST_WARNING, __func__, __VA_ARGS__)
#define st_message(...) shadowtopo_log(ST_MESSAGE, __func__, __VA_ARGS__)
#define st_info(...) shadowtopo_log(ST_INFO, __func__, __VA_ARGS__)
#define st_debug(...) shadowtopo_log(ST_DEBUG, __func__, __VA_ARGS__)

#endif
