// Screen.h — static window state of the host (Screen.h:4-15 / Screen.cpp of the reference).
#pragma once
#include "Vector.h"

class Screen {
public:
    static void setScreenSize(Vector::Vector2 size);
    static Vector::Vector2 getScreenSize();
    static void setWindowPos(Vector::Vector2 pos);
    static Vector::Vector2 getWindowPos();
    static double getDeltaTime();
    static void setDeltaTime(double time);  // ignores 0, as Screen.cpp:35-40
};
