#pragma once
struct half { unsigned short bits; };
namespace Imf { struct Rgba { half r, g, b, a; }; }
