// Screen.cpp — Screen.cpp of the reference: plain static state.
#include "Screen.h"

using Vector::Vector2;

namespace {
Vector2 g_screen_size;
Vector2 g_window_pos;
double g_delta_time = 0.0;
}  // namespace

void Screen::setScreenSize(Vector2 size) { g_screen_size = size; }
Vector2 Screen::getScreenSize() { return g_screen_size; }
void Screen::setWindowPos(Vector2 pos) { g_window_pos = pos; }
Vector2 Screen::getWindowPos() { return g_window_pos; }
double Screen::getDeltaTime() { return g_delta_time; }
void Screen::setDeltaTime(double time) {
    if (time != 0) g_delta_time = time;
}
